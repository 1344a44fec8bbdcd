# Plan tests + full-size parity on the new hashed plan, PMC entries of the
# hashed 8/10/11-generation instances, then the default and driver benches.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sub.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_sub.log; [ $rc -eq 0 ] || exit $rc
CONFIGS="262144x262144:N1:10:1 262144x262144:N1:11:1 262144x262144:N1:8:1" bash scripts/gpu_pmc.sh > gpurun_out/pmc_r2c.log 2>&1
rc=$?; tail -4 gpurun_out/pmc_r2c.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_20.json 2> gpurun_out/bench_20.err
echo "bench20 rc=$?"
