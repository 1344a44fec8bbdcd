# Full GPU suite + smoke, then the rocprofv3 kernel trace/stats of the
# driver's bench command beside the same command unprofiled, then the
# default bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; grep "libgol: dropped" gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r2_prof.sh > gpurun_out/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
echo "bench rc=$?"
