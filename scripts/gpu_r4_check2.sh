#!/bin/bash
# GPU suite (quad child test, diagnostics, degenerate geometry) and smoke on
# the pair-default build, then the quad layout's prefetch-depth A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r4_gpu_suite2.txt 2>&1 &&
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r4_smoke2.txt 2>&1 &&
bash scripts/gpu_r4_quad_pf.sh
