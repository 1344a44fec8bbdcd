#!/bin/bash
# Round 6: tail divisor on the shapes whose bands are 256 / 384 rows.
set -o pipefail
mkdir -p gpurun_out/tail3
T='1,4;1,6;1,8;1,12'
timeout -k 10 200 python -u scripts/band_scan.py 262144x32768 10 160 "$T" > gpurun_out/tail3/262144x32768.txt 2>&1 &&
timeout -k 10 200 python -u scripts/band_scan.py 262144x32768 10 160 "$T" h > gpurun_out/tail3/262144x32768_h.txt 2>&1 &&
timeout -k 10 200 python -u scripts/band_scan.py 131072 10 100 "$T" > gpurun_out/tail3/131072.txt 2>&1 &&
timeout -k 10 200 python -u scripts/band_scan.py 262144x65536 10 100 "$T" > gpurun_out/tail3/262144x65536.txt 2>&1 &&
timeout -k 10 150 python -u scripts/band_scan.py 65536 10 300 "$T" > gpurun_out/tail3/65536.txt 2>&1
