# Round 3 profile of the driver's bench command:
#  1. rocprofv3 --kernel-trace --stats (scripts/prof_summary.py -> profiles/r03_kernel_*)
#  2. rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU over the same command: the
#     PMC clock of the timed launches beside the in-kernel probe clock the same
#     run prints (scripts/clock_reconcile.py -> profiles/r03_clock_reconcile.txt)
#  3. the per-launch PMC table for the depths the bench times at the new bands
#  4. the command unprofiled
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=gpurun_out/prof
C=gpurun_out/clk
mkdir -p $P $C
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/bench_trace -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 > $P/bench_under_rocprof.json 2> $P/bench_under_rocprof.err
rc=$?; echo "rocprof trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 400 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU -T -d $C/bench_clock -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu > $C/bench_under_pmc.json 2> $C/bench_under_pmc.err
rc=$?; echo "rocprof pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
CONFIGS="262144x262144:N1:12:0 262144x262144:N1:8:0 262144x262144:N1:10:1 262144x262144:N1:11:1 262144x262144:N1:8:1" bash scripts/gpu_pmc.sh > gpurun_out/pmc_r3.log 2>&1
rc=$?; tail -3 gpurun_out/pmc_r3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $P/bench.json 2> $P/bench.err
rc=$?; echo "bench rc=$rc"; exit $rc
