#!/bin/bash
# Row-pair-shared B3/S23 circuit (B, in-tree libgol) against the per-row
# circuit (A, ab/rowcirc, -DGOL_PAIR_ROWS=0): parity of B first, then
# alternating depth sweeps at 262144^2 (unhashed and hashed).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
A=$PWD/ab/rowcirc/lib/libgol.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_unhashed_passes.py tests/test_gpu_fullsize.py > gpurun_out/r4_pair_parity.txt 2>&1 || exit 1
for r in 1 2; do
  GOL_LIB_PATH=$A ROUNDS=1 timeout -k 10 120 python scripts/depth_sweep.py 262144 > gpurun_out/r4_pair_sweep.A.$r.txt 2>&1 || exit 1
  ROUNDS=1 timeout -k 10 120 python scripts/depth_sweep.py 262144 > gpurun_out/r4_pair_sweep.B.$r.txt 2>&1 || exit 1
done
GOL_LIB_PATH=$A HASH=1 ROUNDS=1 timeout -k 10 120 python scripts/depth_sweep.py 262144 > gpurun_out/r4_pair_sweep_hash.A.txt 2>&1 &&
HASH=1 ROUNDS=1 timeout -k 10 120 python scripts/depth_sweep.py 262144 > gpurun_out/r4_pair_sweep_hash.B.txt 2>&1
