#!/bin/bash
# Round-4 final build: the whole GPU suite, smoke(), the driver's bench
# command (with the CPU leg) and the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r4_final_suite.txt 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_final_smoke.txt 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4_final_bench.json 2> gpurun_out/r4_final_bench.err || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/r4_final_bench_default.json 2> gpurun_out/r4_final_bench_default.err
