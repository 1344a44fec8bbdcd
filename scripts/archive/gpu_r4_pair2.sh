#!/bin/bash
# Pair-row build (occupancy unforced, quads per-row): quad and hashed parity,
# then the depth sweeps behind the pass planner's cost table, and the per-row
# build (ab/rowcirc) at 262144^2 on the same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
A=$PWD/ab/rowcirc/lib/libgol.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_quads.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py > gpurun_out/r4_pair2_parity.txt 2>&1 || exit 1
ROUNDS=3 timeout -k 10 200 python scripts/depth_sweep.py 262144 262144x32768 65536 > gpurun_out/r4_pair2_sweep.B.txt 2>&1 || exit 1
HASH=1 ROUNDS=3 timeout -k 10 200 python scripts/depth_sweep.py 262144 65536 > gpurun_out/r4_pair2_sweep_hash.B.txt 2>&1 || exit 1
GOL_LIB_PATH=$A ROUNDS=3 timeout -k 10 200 python scripts/depth_sweep.py 262144 65536 > gpurun_out/r4_pair2_sweep.A.txt 2>&1 || exit 1
GOL_LIB_PATH=$A HASH=1 ROUNDS=3 timeout -k 10 200 python scripts/depth_sweep.py 262144 65536 > gpurun_out/r4_pair2_sweep_hash.A.txt 2>&1
