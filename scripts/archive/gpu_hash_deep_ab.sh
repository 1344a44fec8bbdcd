# Same-box A/B: ab/old (HEAD: hashed passes peeled only up to G = 9, hashed
# G >= 10 at 2 waves) vs the working tree (row step force-inlined, hashed
# G = 10..12 peeled at 3 waves): hashed depth sweep G = 6..12 and hashed /
# unhashed pass mixes at 262144^2.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/hash_deep_ab.log
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then L=$PWD/ab/old/lib/libgol.so; else L=$PWD/akka-game-of-life_amd/lib/libgol.so; fi
    GOL_LIB_PATH=$L HASH=1 ROUNDS=1 MAXG=12 timeout -k 10 200 python scripts/depth_sweep.py 262144x262144 65536x65536 2>&1 | grep -E "G=(6|7|8|9|10|11|12) " | sed "s/^/$v r$r /" >> gpurun_out/hash_deep_ab.log || exit 1
    GOL_LIB_PATH=$L timeout -k 10 200 python scripts/plan_mix_ab.py --rounds 2 --hash 12,8 10,10 11,9 7,7,6 8,6,6 2>&1 | grep best | sed "s/^/$v r$r /" >> gpurun_out/hash_deep_ab.log || exit 1
    GOL_LIB_PATH=$L timeout -k 10 200 python scripts/plan_mix_ab.py --rounds 2 12,8 12,12,12,12,12 2>&1 | grep best | sed "s/^/$v r$r /" >> gpurun_out/hash_deep_ab.log || exit 1
  done
done
cat gpurun_out/hash_deep_ab.log
