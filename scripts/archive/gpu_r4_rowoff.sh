#!/bin/bash
# Row addressing by plane offsets (B, in-tree: no per-row argument s_load,
# 32 x 32-bit pitch products) vs the pointer select (A, ab/rowptr,
# -DGOL_ROW_OFF=0): parity of B at the bench's sizes, then the driver's
# command alternating A / B three times on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
A=$PWD/ab/rowptr/lib/libgol.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py tests/test_gpu_unhashed_passes.py tests/test_gpu_rccl.py > gpurun_out/r4_rowoff_parity.txt 2>&1 || exit 1
for r in 1 2 3; do
  GOL_LIB_PATH=$A timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r4_rowoff.A$r.json 2> gpurun_out/r4_rowoff.A$r.err || exit 1
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r4_rowoff.B$r.json 2> gpurun_out/r4_rowoff.B$r.err || exit 1
done
