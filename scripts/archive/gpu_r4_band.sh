#!/bin/bash
# Band heights for the pair kernels' G = 10 passes on the two shapes whose
# pass is only 1-2 rounds of resident waves: 65536^2 (17 strips, the bench's
# secondary) and one N = 8 rank's shard (262144 x 32768, self-ring).  Band 0
# = the library's choice; the tail split on for every config (GOL_TAIL).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
GOL_TAIL=1.0,3 timeout -k 10 300 python scripts/band_ab.py --shape 65536x65536 --rounds 4 \
  10:0,10:0 10:192,10:192 10:160,10:160 10:128,10:128 10:96,10:96 > gpurun_out/r4_band_65536.txt 2>&1 || exit 1
GOL_TAIL=1.0,3 timeout -k 10 300 python scripts/band_ab.py --shape 262144x32768 --ring --rounds 4 \
  10:0,10:0 10:512,10:512 10:384,10:384 10:256,10:256 10:192,10:192 > gpurun_out/r4_band_32768.txt 2>&1
