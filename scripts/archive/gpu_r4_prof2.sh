#!/bin/bash
# Round 4 profile of the pair-row build: the driver's bench command (torch-free bench.py):
#  1. rocprofv3 --kernel-trace --stats  (scripts/prof_summary.py -> profiles/r04_kernel_*)
#  2. rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU over the same command (clock reconcile)
#  3. the per-launch PMC table for the depths the bench times (profiles/pmc_launch.json)
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
CONFIGS="262144x262144:N1:10:0 262144x262144:N1:10:1 65536x65536:N1:10:0 65536x65536:N1:7:0 65536x65536:N1:1:0 262144x32768:ring:10:0" bash scripts/gpu_pmc.sh > gpurun_out/pmc_r4p.log 2>&1
rc=$?; tail -3 gpurun_out/pmc_r4p.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $P/bench.json 2> $P/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > $P/bench_default.json 2> $P/bench_default.err
rc=$?; echo "bench default rc=$rc"; exit $rc
