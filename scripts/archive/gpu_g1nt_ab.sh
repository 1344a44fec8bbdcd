# Same-box A/B: single-generation passes with plain vs non-temporal stores
# (ab/ntg1: -DGOL_G1_NT_STORES=1, step_kernel only), 3 interleaved rounds.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/g1nt_ab.log
for r in 1 2 3; do
  for v in cur nt; do
    if [ $v = nt ]; then L=$PWD/ab/ntg1/lib/libgol.so; else L=$PWD/akka-game-of-life_amd/lib/libgol.so; fi
    for shape in 65536x65536 262144x262144 262144x32768; do
      GOL_LIB_PATH=$L GPPS=1 BANDS=0 TAILS=";" ROUNDS=1 GENS=64 timeout -k 10 120 python scripts/rank_sweep.py $shape 2>&1 | grep shape= | sed "s/^/$v r$r /" >> gpurun_out/g1nt_ab.log || exit 1
    done
  done
done
cat gpurun_out/g1nt_ab.log
