# Round 3 final rehearsal on a fresh box: rocprofv3 kernel trace + stats of
# the driver's bench command, one GRBM_GUI_ACTIVE / SQ_INSTS_VALU pass of it
# (clock reconciliation), the GPU suite, smoke(), the default bench and the
# driver's command unprofiled.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=gpurun_out/prof
C=gpurun_out/clk
mkdir -p $P $C
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/bench_trace -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 > $P/bench_under_rocprof.json 2> $P/bench_under_rocprof.err
rc=$?; echo "rocprof trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 400 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU -T -d $C/bench_clock -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu > $C/bench_under_pmc.json 2> $C/bench_under_pmc.err
rc=$?; echo "rocprof pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_final4_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r3_final4_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3_final4_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/r3_final4_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r3_final4_bench_default.json 2> gpurun_out/r3_final4_bench_default.err
rc=$?; echo "bench default rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $P/bench.json 2> $P/bench.err
rc=$?; echo "bench driver rc=$rc"; exit $rc
