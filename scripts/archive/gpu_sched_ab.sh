# Same-box A/B: ab/old = default scheduler, ab/new = -amdgpu-sched-strategy=max-ilp
# (same sources): depth sweeps and the bench's pass mixes.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/sched_ab.log
for r in 1 2; do
  for v in old new; do
    GOL_LIB_PATH=$PWD/ab/$v/lib/libgol.so ROUNDS=2 MAXG=12 timeout -k 10 200 python scripts/depth_sweep.py 262144x262144 65536x65536 2>&1 | grep -E "G=(6|8|10|12) " | sed "s/^/$v r$r /" >> gpurun_out/sched_ab.log || exit 1
    GOL_LIB_PATH=$PWD/ab/$v/lib/libgol.so HASH=1 ROUNDS=2 MAXG=8 timeout -k 10 200 python scripts/depth_sweep.py 262144x262144 2>&1 | grep -E "G=(6|7|8) " | sed "s/^/$v r$r /" >> gpurun_out/sched_ab.log || exit 1
    GOL_LIB_PATH=$PWD/ab/$v/lib/libgol.so timeout -k 10 200 python scripts/plan_mix_ab.py --rounds 2 12,8 12,12,12,12,12 2>&1 | grep best | sed "s/^/$v r$r /" >> gpurun_out/sched_ab.log || exit 1
  done
done
cat gpurun_out/sched_ab.log
