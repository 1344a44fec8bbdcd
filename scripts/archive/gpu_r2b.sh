# GPU suite (HIP runtime error log on), smoke, default bench, the driver's
# bench command, then the per-rank band sweep at 8-12 generations per pass.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AMD_LOG_LEVEL=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; grep -n "libgol: dropped\|:1:" gpurun_out/pytest_gpu.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_20.json 2> gpurun_out/bench_20.err
rc=$?; echo "bench20 rc=$rc"; [ $rc -eq 0 ] || exit $rc
BANDS=0,256,384,512,640,728 TAILS=";0,0" GPPS=8,10,12 ROUNDS=2 GENS=48 timeout -k 10 300 python scripts/rank_sweep.py 262144x32768 --ring > gpurun_out/r2b_rank_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; [ $rc -eq 0 ] || exit $rc
BANDS=0 TAILS=";0,0" GPPS=8,12 ROUNDS=2 GENS=48 timeout -k 10 300 python scripts/rank_sweep.py 262144x262144 --ring > gpurun_out/r2b_whole_sweep.log 2>&1
echo "whole rc=$?"
