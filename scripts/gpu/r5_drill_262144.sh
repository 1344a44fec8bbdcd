#!/bin/bash
# Round 5: the bench's N = 8 fault drill at 262144^2 as eight loopback ranks on one GPU.
set -o pipefail
mkdir -p gpurun_out
df -h /tmp /dev/shm > gpurun_out/r5_drill_262144.txt 2>&1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread \
    "tests/test_gpu_fault_drill.py::test_fault_drill_loopback_262144_golden" >> gpurun_out/r5_drill_262144.txt 2>&1
rc=$?
tail -8 gpurun_out/r5_drill_262144.txt
exit $rc
