# GPU tests on the in-tree build, then same-box A/B of ab/old vs ab/new
# (scripts/ab_build.sh): pair-layout horizontal-first kernel at G = 6, 7 and
# the vertical-first kernel at 16-byte lanes, G = 6.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
GPPS=6,7 VECS=2 bash scripts/gpu_ab.sh > gpurun_out/ab_circuit_vec2.txt 2>&1 || exit $?
GPPS=6 VECS=4 bash scripts/gpu_ab.sh > gpurun_out/ab_circuit_vec4.txt 2>&1 || exit $?
cat gpurun_out/ab_circuit_vec2.txt gpurun_out/ab_circuit_vec4.txt
