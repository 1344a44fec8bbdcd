#!/bin/bash
# Quad vs pair layout A/B on one box (scripts/quad_ab.py), alternating twice,
# then the quad layout's depth sweep (pass planner costs), unhashed and hashed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2; do
  for m in pairs quads; do
    timeout -k 10 180 python scripts/quad_ab.py $m gpurun_out/r4_quad_ab.$m.$r.json > gpurun_out/r4_quad_ab.$m.$r.log 2>&1 || exit 1
  done
done
ROUNDS=2 timeout -k 10 240 python scripts/depth_sweep.py 262144 262144x32768 65536 > gpurun_out/r4_depth_sweep_quads.txt 2>&1 &&
HASH=1 ROUNDS=2 timeout -k 10 240 python scripts/depth_sweep.py 262144 65536 > gpurun_out/r4_depth_sweep_quads_hash.txt 2>&1
