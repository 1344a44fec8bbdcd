#!/bin/bash
# Round 4 GPU check: the GPU suite, smoke, the driver's bench command, and the
# VERDICT r03 item-3 micro-benchmark (scripts/micro/valu_rate VALU_RATE_R4).
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r4_gpu_suite.txt 2>&1 &&
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r4_smoke.txt 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_bench_driver.json \
    2> gpurun_out/r4_bench_driver.err &&
VALU_RATE_R4=1 timeout -k 10 120 scripts/micro/valu_rate > gpurun_out/r4_valu_mix.txt 2>&1
