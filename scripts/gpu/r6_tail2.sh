#!/bin/bash
# Round 6: tail-split divisor on the hashed passes and at G = 7 / 12.
set -o pipefail
mkdir -p gpurun_out/tail2
T='1,3;1,4;1,5'
timeout -k 10 150 python -u scripts/band_scan.py 65536 7 301 "$T" h > gpurun_out/tail2/65536_g7h.txt 2>&1 &&
timeout -k 10 300 python -u scripts/band_scan.py 262144 10 30 "$T" h > gpurun_out/tail2/262144_g10h.txt 2>&1 &&
timeout -k 10 150 python -u scripts/band_scan.py 65536 10 300 "$T" h > gpurun_out/tail2/65536_g10h.txt 2>&1 &&
timeout -k 10 300 python -u scripts/band_scan.py 262144 12 36 "$T" > gpurun_out/tail2/262144_g12.txt 2>&1 &&
timeout -k 10 200 python -u scripts/band_scan.py 262144x32768 10 160 "$T" h > gpurun_out/tail2/262144x32768_g10h.txt 2>&1
