# Single-generation passes: XCD chunk (blocks kept on one XCD) sweep, 2 rounds.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/g1_xcd.log
for r in 1 2; do
  for c in 8 16 32 64; do
    for shape in 65536x65536 262144x262144 262144x32768; do
      GOL_XCD_CHUNK=$c GPPS=1 BANDS=0 TAILS=";" ROUNDS=1 GENS=64 timeout -k 10 120 python scripts/rank_sweep.py $shape 2>&1 | grep shape= | sed "s/^/chunk=$c r$r /" >> gpurun_out/g1_xcd.log || exit 1
    done
  done
done
cat gpurun_out/g1_xcd.log
