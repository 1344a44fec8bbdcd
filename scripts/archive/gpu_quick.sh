# GPU tests, then the bench (no CPU baseline) and a short sweep of pass depth.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_quick.json
[ $rc -eq 0 ] || exit $rc
VECS=2 GPPS=${GPPS:-4,5,6,7,8} BANDS=0 HASH=0 ROUNDS=3 timeout -k 10 300 python scripts/tune.py 262144 65536 262144x32768 > gpurun_out/tune_quick.log 2>&1
rc=$?; echo "tune rc=$rc"; cat gpurun_out/tune_quick.log
exit $rc
