#!/bin/bash
# Round 5, VERDICT r04 item 3: price the fused hash on the pair-row loop mix
# (scripts/micro/valu_rate.hip, VALU_RATE_HASH).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
VALU_RATE_HASH=1 timeout -k 10 120 scripts/micro/valu_rate > gpurun_out/r5_hash_micro.txt 2>&1
rc=$?
cat gpurun_out/r5_hash_micro.txt
exit $rc
