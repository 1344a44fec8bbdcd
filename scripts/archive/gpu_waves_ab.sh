# Same-box A/B (ab/old = HEAD, ab/new = forced 4 waves/SIMD for hashed G = 9
# and unhashed G = 10, with small spills): depth sweeps G = 8..12.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/waves_ab.log
for r in 1 2; do
  for v in old new; do
    GOL_LIB_PATH=$PWD/ab/$v/lib/libgol.so ROUNDS=2 MAXG=12 timeout -k 10 200 python scripts/depth_sweep.py 262144x262144 262144x32768 2>&1 | grep -E "G=(8|9|10|11|12) " | sed "s/^/$v r$r /" >> gpurun_out/waves_ab.log || exit 1
    GOL_LIB_PATH=$PWD/ab/$v/lib/libgol.so HASH=1 ROUNDS=2 MAXG=10 timeout -k 10 200 python scripts/depth_sweep.py 262144x262144 65536x65536 2>&1 | grep -E "G=(7|8|9|10) " | sed "s/^/$v r$r /" >> gpurun_out/waves_ab.log || exit 1
  done
done
cat gpurun_out/waves_ab.log
