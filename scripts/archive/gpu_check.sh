cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --maxfail=15 > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -40 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 5 > gpurun_out/bench.log 2>&1
  echo "bench rc=$?"
  tail -5 gpurun_out/bench.log
fi
