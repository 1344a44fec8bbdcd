# Per-rank ring schedule: wall vs kernel time with and without the 1-rank
# RCCL self-ring (scripts/rank_sweep.py), and a rocprofv3 kernel trace of the
# ring run (interior launch, boundary launch, RCCL kernels per pass).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ring
GPPS=12,8 BANDS=0 TAILS="" ROUNDS=3 GENS=48 timeout -k 10 200 python scripts/rank_sweep.py 262144x32768 > gpurun_out/ring/sweep.log 2>&1 || exit $?
GPPS=12,8 BANDS=0 TAILS="" ROUNDS=3 GENS=48 timeout -k 10 200 python scripts/rank_sweep.py 262144x32768 --ring >> gpurun_out/ring/sweep.log 2>&1 || exit $?
cat gpurun_out/ring/sweep.log
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/ring/trace -o run --output-format csv -- python3 scripts/prof_run.py 262144x32768 12 --passes 8 --ring > gpurun_out/ring/trace.log 2>&1
echo "trace rc=$?"
