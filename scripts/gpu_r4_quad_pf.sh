#!/bin/bash
# Quad layout: prefetch depth 2 (in-tree build) / 3 / 4 (ab/ builds), against
# the pair layout, same box, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 180 python scripts/quad_ab.py pairs gpurun_out/r4_quad_pf.pairs.$r.json > gpurun_out/r4_quad_pf.pairs.$r.log 2>&1 || exit 1
  timeout -k 10 180 python scripts/quad_ab.py quads gpurun_out/r4_quad_pf.pf2.$r.json > gpurun_out/r4_quad_pf.pf2.$r.log 2>&1 || exit 1
  for v in pf3 pf4; do
    GOL_LIB_PATH=$PWD/ab/$v/lib/libgol.so timeout -k 10 180 python scripts/quad_ab.py quads gpurun_out/r4_quad_pf.$v.$r.json > gpurun_out/r4_quad_pf.$v.$r.log 2>&1 || exit 1
  done
done
