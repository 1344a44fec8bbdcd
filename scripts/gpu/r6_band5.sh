#!/bin/bash
# Round 6: band heights under the new tail rule on the N = 8 shard shape and
# 131072^2 (256- / 384-row automatic bands).
set -o pipefail
mkdir -p gpurun_out/band5
timeout -k 10 300 python -u scripts/band_scan.py 262144x32768 10 160 '192@1,6;320@1,6;384@1,6;448@1,6;512@1,6;512@1,4;640@1,4;256@0.75,6;256@1.5,6' > gpurun_out/band5/262144x32768.txt 2>&1 &&
timeout -k 10 300 python -u scripts/band_scan.py 131072 10 100 '256@1,6;320@1,6;448@1,6;512@1,6;512@1,4;640@1,4;768@1,4;384@0.75,6;384@1.5,6' > gpurun_out/band5/131072.txt 2>&1
