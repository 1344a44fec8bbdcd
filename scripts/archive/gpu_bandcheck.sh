cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VECS=0 GPPS=6 BANDS=0,256 HASH=0 ROUNDS=3 timeout -k 10 600 python scripts/tune.py 262144 262144x131072 262144x65536 262144x32768 65536 > gpurun_out/bandcheck.log 2>&1
echo "rc=$?"; cat gpurun_out/bandcheck.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench4.json 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/bench4.json
