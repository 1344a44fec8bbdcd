# Single-generation parity on the new default (nt stores at G = 1), the G = 1
# PMC entry, then a same-box A/B of non-temporal stores in every kernel
# (ab/ntall: -DGOL_NT_STORES=1) on the planner's multi-generation passes.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rccl.py tests/test_gpu_group.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sub.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_sub.log; [ $rc -eq 0 ] || exit $rc
CONFIGS="65536x65536:N1:1:0 262144x262144:N1:1:0" bash scripts/gpu_pmc.sh > gpurun_out/pmc_g1.log 2>&1
rc=$?; tail -3 gpurun_out/pmc_g1.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/ntall_ab.log
for r in 1 2; do
  for v in cur nt; do
    if [ $v = nt ]; then L=$PWD/ab/ntall/lib/libgol.so; else L=$PWD/akka-game-of-life_amd/lib/libgol.so; fi
    GOL_LIB_PATH=$L timeout -k 10 200 python scripts/plan_mix_ab.py --rounds 2 12,8 12,12,12,12,12 2>&1 | grep best | sed "s/^/$v r$r /" >> gpurun_out/ntall_ab.log || exit 1
    GOL_LIB_PATH=$L GPPS=8,12 BANDS=0 TAILS=";" ROUNDS=1 GENS=48 timeout -k 10 120 python scripts/rank_sweep.py 65536x65536 2>&1 | grep shape= | sed "s/^/$v r$r /" >> gpurun_out/ntall_ab.log || exit 1
    GOL_LIB_PATH=$L GPPS=12 BANDS=0 TAILS=";" ROUNDS=1 GENS=48 timeout -k 10 120 python scripts/rank_sweep.py 262144x32768 --ring 2>&1 | grep shape= | sed "s/^/$v r$r /" >> gpurun_out/ntall_ab.log || exit 1
  done
done
cat gpurun_out/ntall_ab.log
