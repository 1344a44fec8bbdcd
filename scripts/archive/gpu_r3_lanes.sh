# Round 3: switch off the lanes past the last strip's halo lane in unhashed
# multi-generation passes (GOL_IDLE_LANES_OFF).  Parity (unhashed passes at
# every depth and strip remainder, the parity and full-size suites), then a
# same-box A/B of the driver's bench command against -DGOL_IDLE_LANES_OFF=0.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_unhashed_passes.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
    tests/test_gpu_group.py tests/test_gpu_rccl.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_lanes_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3_lanes_tests.log; [ $rc -eq 0 ] || exit $rc
AB="lanes_on lanes_off" ROUNDS=4 bash scripts/gpu_ab_bench.sh > gpurun_out/r3_lanes_ab.txt 2>&1
rc=$?; cat gpurun_out/r3_lanes_ab.txt; exit $rc
