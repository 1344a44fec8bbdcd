# Round 3 round-end rehearsal after the idle-lanes change, on a fresh box:
# the GPU suite, smoke(), the default bench and the driver's command (its
# line also serves profiles/r03_kernel_trace.txt as the unprofiled run).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_final2_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r3_final2_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3_final2_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/r3_final2_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r3_final2_bench_default.json 2> gpurun_out/r3_final2_bench_default.err
rc=$?; echo "bench default rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err
rc=$?; echo "bench driver rc=$rc"; exit $rc
