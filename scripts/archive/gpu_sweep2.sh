cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VECS=4 GPPS=6,7,8 BANDS=192,256,384,512,768 HASH=1 ROUNDS=3 timeout -k 10 600 python scripts/tune.py 262144 > gpurun_out/sweep2.log 2>&1
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/sweep2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --hash --no-cpu > gpurun_out/bench_hash.json 2>&1; echo "bench-hash rc=$?"; tail -1 gpurun_out/bench_hash.json
