#!/bin/bash
# Row loop without the per-row multi-wrap branch (B, in-tree: one basic block
# per 6-row unroll) vs HEAD (A, ab/head): parity of B, then the driver's
# command alternating A / B three times on one box, then B's depth sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
A=$PWD/ab/head/lib/libgol.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_unhashed_passes.py tests/test_gpu_known_answers.py > gpurun_out/r4_nb_parity.txt 2>&1 || exit 1
for r in 1 2 3; do
  GOL_LIB_PATH=$A timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r4_nb.A$r.json 2> gpurun_out/r4_nb.A$r.err || exit 1
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r4_nb.B$r.json 2> gpurun_out/r4_nb.B$r.err || exit 1
done
ROUNDS=2 timeout -k 10 200 python scripts/depth_sweep.py 262144 65536 > gpurun_out/r4_nb_sweep.B.txt 2>&1 &&
GOL_LIB_PATH=$A ROUNDS=2 timeout -k 10 200 python scripts/depth_sweep.py 262144 65536 > gpurun_out/r4_nb_sweep.A.txt 2>&1
