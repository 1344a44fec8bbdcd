#!/bin/bash
# Pair-row build: the whole GPU suite, then the driver's bench command on B
# (in-tree) and A (ab/rowcirc, per-row circuit, its own planner table),
# alternating, and B's default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
A=$PWD/ab/rowcirc/lib/libgol.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r4_pair3_suite.txt 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4_pair3_bench.B1.json 2> gpurun_out/r4_pair3_bench.B1.err || exit 1
GOL_LIB_PATH=$A timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r4_pair3_bench.A1.json 2> gpurun_out/r4_pair3_bench.A1.err || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r4_pair3_bench.B2.json 2> gpurun_out/r4_pair3_bench.B2.err || exit 1
GOL_LIB_PATH=$A timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r4_pair3_bench.A2.json 2> gpurun_out/r4_pair3_bench.A2.err || exit 1
timeout -k 10 300 python3 bench.py --no-cpu > gpurun_out/r4_pair3_bench.Bdefault.json 2> gpurun_out/r4_pair3_bench.Bdefault.err
