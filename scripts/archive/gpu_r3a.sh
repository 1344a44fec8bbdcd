# Round 3, first GPU pass: the new parity / status / fault tests, the whole
# GPU suite, then the driver's bench command (parity against the golden table).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "hip_status or unhashed_single or config5 or in_flight or snapshot_query" > gpurun_out/r3a_new.log 2>&1
rc=$?; tail -5 gpurun_out/r3a_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "not (hip_status or unhashed_single or config5 or in_flight or snapshot_query)" > gpurun_out/r3a_suite.log 2>&1
rc=$?; tail -5 gpurun_out/r3a_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r3a_bench20.json 2> gpurun_out/r3a_bench20.err
rc=$?; cat gpurun_out/r3a_bench20.json; exit $rc
