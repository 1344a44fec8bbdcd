#!/bin/bash
# Round 5: the fault-drill and elastic GPU tests after the light-cone reader change.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_fault_drill.py tests/test_elastic.py -m gpu > gpurun_out/r5_drill_check.txt 2>&1
rc=$?
tail -5 gpurun_out/r5_drill_check.txt
exit $rc
