# GPU tests, then same-box A/B of the fused-hash kernels (ab/hbase = HEAD).
cd $GRAFT_REPO_ROOT
O=gpurun_out/hash
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for v in hbase new; do
    lib=$PWD/akka-game-of-life_amd/lib/libgol.so; [ $v = hbase ] && lib=$PWD/ab/hbase/lib/libgol.so
    GOL_LIB_PATH=$lib VECS=0 GPPS=6 BANDS=0 HASH=1 ROUNDS=2 \
      timeout -k 10 200 python scripts/tune.py 262144 65536 > $O/ab_$v.$round.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "ab $v rc=$rc"; tail -5 $O/ab_$v.$round.log; exit $rc; }
    sed "s/^/$v r$round /" $O/ab_$v.$round.log | cut -c1-60,150-
  done
done
