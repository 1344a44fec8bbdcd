cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
GOL_STENCIL_VARIANT=2 timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py -m gpu -q -p no:cacheprovider --maxfail=5 -x > gpurun_out/pytest_v2.log 2>&1
rc=$?; echo "pytest v2 rc=$rc"; tail -5 gpurun_out/pytest_v2.log
[ $rc -eq 0 ] || exit $rc
for v in 1 2; do
  GOL_STENCIL_VARIANT=$v VECS=2,4 GPPS=4,6,8 BANDS=0,256 HASH=0 ROUNDS=3 timeout -k 10 300 python scripts/tune.py 262144 65536 > gpurun_out/var$v.log 2>&1
  echo "variant $v rc=$?"; sed "s/^/v$v /" gpurun_out/var$v.log
done
