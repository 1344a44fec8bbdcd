# Same-box A/B of library builds (ab/old, ab/new) on the hashed depth sweep
# at 262144^2 and 65536^2 (G = 6..10) and the bench's hashed pass mixes.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/hash_peel_ab.log
for r in 1 2; do
  for v in old new; do
    GOL_LIB_PATH=$PWD/ab/$v/lib/libgol.so HASH=1 ROUNDS=2 MAXG=10 timeout -k 10 200 python scripts/depth_sweep.py 262144x262144 65536x65536 2>&1 | grep -E "G=(6|7|8|9|10) " | sed "s/^/$v r$r /" >> gpurun_out/hash_peel_ab.log || exit 1
    GOL_LIB_PATH=$PWD/ab/$v/lib/libgol.so timeout -k 10 200 python scripts/plan_mix_ab.py --rounds 2 --hash 10,10 8,12 6,6,8 8,8,4 12,8 2>&1 | grep best | sed "s/^/$v r$r /" >> gpurun_out/hash_peel_ab.log || exit 1
  done
done
cat gpurun_out/hash_peel_ab.log
