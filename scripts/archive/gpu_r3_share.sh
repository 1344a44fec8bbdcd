# Round 3: shared edge lanes (63-pair strips for unhashed multi-generation
# passes).  Parity first (new edge-lane tests + the suites whose unhashed
# passes now run them), then a same-box A/B of the driver's bench command
# against a build with -DGOL_SHARE_HALO=0 (ab/noshare), interleaved rounds.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_unhashed_passes.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
    tests/test_gpu_rccl.py tests/test_gpu_group.py tests/test_gpu_loopback.py tests/test_gpu_snapshot.py \
    -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_share_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3_share_tests.log; [ $rc -eq 0 ] || exit $rc
AB="noshare share" ROUNDS=3 bash scripts/gpu_ab_bench.sh > gpurun_out/r3_share_ab.txt 2>&1
rc=$?; cat gpurun_out/r3_share_ab.txt; exit $rc
