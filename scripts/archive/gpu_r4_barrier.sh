#!/bin/bash
# Scheduling barrier after every n-th stage of a row (unhashed instances,
# -DGOL_STAGE_BARRIER=n, ab/bar*) vs none (shipped, in-tree): the driver's
# command, alternating, two rounds, one box; quick parity of each variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in 1 2 5; do
  GOL_LIB_PATH=$PWD/ab/bar$v/lib/libgol.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_unhashed_passes.py tests/test_gpu_known_answers.py > gpurun_out/r4_bar$v.parity.txt 2>&1 || exit 1
done
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r4_bar.none$r.json 2> gpurun_out/r4_bar.none$r.err || exit 1
  for v in 1 2 5; do
    GOL_LIB_PATH=$PWD/ab/bar$v/lib/libgol.so timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r4_bar.b$v.$r.json 2> gpurun_out/r4_bar.b$v.$r.err || exit 1
  done
done
