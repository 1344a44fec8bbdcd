#!/bin/bash
# GPU suite (quad child test, diagnostics, degenerate geometry) and smoke,
# then the round-4 profile of the driver's bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r4_gpu_suite2.txt 2>&1 &&
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r4_smoke2.txt 2>&1 &&
bash scripts/gpu_r4_prof.sh > gpurun_out/r4_prof.log 2>&1
