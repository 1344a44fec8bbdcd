cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VECS=1,2 GPPS=5,6,7 BANDS=0,128,192,256,384 HASH=0 ROUNDS=3 timeout -k 10 600 python scripts/tune.py 262144 65536 > gpurun_out/sweep3.log 2>&1
echo "sweep rc=$?"; cat gpurun_out/sweep3.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench3.json 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/bench3.json
timeout -k 10 300 python bench.py --no-cpu --no-secondary --hash > gpurun_out/bench3h.json 2>&1; echo "bench-hash rc=$?"; tail -1 gpurun_out/bench3h.json
