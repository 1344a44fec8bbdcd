# Same-box A/B: 4-wave workgroups (default) vs 1-wave workgroups
# (ab/wg1: -DGOL_WAVES_PER_WG=1; XCD chunk 8 and 32 blocks), pass mixes at
# 262144^2 and per-generation times at 65536^2 and the per-rank self-ring.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/wg_ab.log
for r in 1 2; do
  for v in wg4 wg1c8 wg1c32; do
    case $v in
      wg4) L=$PWD/akka-game-of-life_amd/lib/libgol.so; C=8;;
      wg1c8) L=$PWD/ab/wg1/lib/libgol.so; C=8;;
      wg1c32) L=$PWD/ab/wg1/lib/libgol.so; C=32;;
    esac
    GOL_LIB_PATH=$L GOL_XCD_CHUNK=$C timeout -k 10 200 python scripts/plan_mix_ab.py --rounds 2 12,8 12,12,12,12,12 2>&1 | grep best | sed "s/^/$v r$r /" >> gpurun_out/wg_ab.log || exit 1
    GOL_LIB_PATH=$L GOL_XCD_CHUNK=$C GPPS=8 BANDS=0 TAILS=";" ROUNDS=1 GENS=96 timeout -k 10 120 python scripts/rank_sweep.py 65536x65536 2>&1 | grep shape= | sed "s/^/$v r$r /" >> gpurun_out/wg_ab.log || exit 1
    GOL_LIB_PATH=$L GOL_XCD_CHUNK=$C GPPS=12 BANDS=0 TAILS=";" ROUNDS=1 GENS=48 timeout -k 10 120 python scripts/rank_sweep.py 262144x32768 --ring 2>&1 | grep shape= | sed "s/^/$v r$r /" >> gpurun_out/wg_ab.log || exit 1
  done
done
cat gpurun_out/wg_ab.log
