cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --maxfail=5 > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -eq 0 ]; then
  VECS=2,4 GPPS=1,2,4,5,6,7,8 BANDS=0,32,64,128,256 HASH=0 timeout -k 10 900 python scripts/tune.py > gpurun_out/tune.log 2>&1
  echo "tune rc=$?"; cat gpurun_out/tune.log
fi
