# Round 3, after the idle-lanes change: refresh the per-launch PMC keys the
# bench reads for unhashed passes over rows with a partial last strip, then
# profile the driver's bench command (rocprofv3 kernel trace + stats; one
# GRBM_GUI_ACTIVE / SQ_INSTS_VALU pass for the clock reconciliation).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=gpurun_out/prof
C=gpurun_out/clk
mkdir -p $P $C
CONFIGS="262144x262144:N1:12:0 262144x262144:N1:8:0 65536x65536:N1:8:0 262144x32768:ring:12:0 262144x32768:ring:8:0" \
    bash scripts/gpu_pmc.sh > gpurun_out/pmc_r3c.log 2>&1
rc=$?; tail -2 gpurun_out/pmc_r3c.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/bench_trace -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 > $P/bench_under_rocprof.json 2> $P/bench_under_rocprof.err
rc=$?; echo "rocprof trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 400 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU -T -d $C/bench_clock -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu > $C/bench_under_pmc.json 2> $C/bench_under_pmc.err
rc=$?; echo "rocprof pmc rc=$rc"; exit $rc
