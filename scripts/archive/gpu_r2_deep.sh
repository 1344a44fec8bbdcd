# Round 2, 12-generation passes: GPU test suite, then the per-launch PMC
# passes for the depths the bench's plans now use (scripts/gpu_pmc.sh).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
CONFIGS="262144x262144:N1:12:0 262144x262144:N1:10:1 262144x32768:N1:12:0 262144x32768:ring:12:0 262144x65536:ring:12:0 262144x131072:ring:12:0 262144x262144:ring:12:0 262144x262144:ring:8:0" bash scripts/gpu_pmc.sh > gpurun_out/pmc.log 2>&1
rc=$?; tail -12 gpurun_out/pmc.log; exit $rc
