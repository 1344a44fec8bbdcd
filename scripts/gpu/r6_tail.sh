#!/bin/bash
# Round 6: tail-split divisor / fraction at G = 10 across shapes (automatic
# bands), scored per probed GHz (scripts/band_scan.py).
set -o pipefail
mkdir -p gpurun_out/tail
T='1,3;1,4;1,5;1,6;1,8;0.75,4;1.5,4;2,4;0.5,4'
timeout -k 10 150 python -u scripts/band_scan.py 65536 10 300 "$T" > gpurun_out/tail/65536.txt 2>&1 &&
timeout -k 10 200 python -u scripts/band_scan.py 262144x32768 10 160 "$T" > gpurun_out/tail/262144x32768.txt 2>&1 &&
timeout -k 10 200 python -u scripts/band_scan.py 131072 10 100 "$T" > gpurun_out/tail/131072.txt 2>&1 &&
timeout -k 10 300 python -u scripts/band_scan.py 262144 10 30 "$T" > gpurun_out/tail/262144.txt 2>&1
