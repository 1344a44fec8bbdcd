cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --maxfail=5 > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -eq 0 ]; then
  BANDS=0,64,128,256,512 timeout -k 10 600 python scripts/tune.py > gpurun_out/tune.log 2>&1
  echo "tune rc=$?"; cat gpurun_out/tune.log
fi
