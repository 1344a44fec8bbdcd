#!/bin/bash
# Round 6: the band-dependent tail divisor (default "-") against /4 and /3,
# then the GPU suite.
set -o pipefail
mkdir -p gpurun_out/tail4
T='1,4;1,3'
timeout -k 10 300 python -u scripts/band_scan.py 262144 10 30 "$T" > gpurun_out/tail4/262144.txt 2>&1 &&
timeout -k 10 200 python -u scripts/band_scan.py 262144x32768 10 160 "$T" > gpurun_out/tail4/262144x32768.txt 2>&1 &&
timeout -k 10 200 python -u scripts/band_scan.py 131072 10 100 "$T" > gpurun_out/tail4/131072.txt 2>&1 &&
timeout -k 10 150 python -u scripts/band_scan.py 65536 10 300 "$T" > gpurun_out/tail4/65536.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/tail4/suite.txt 2>&1
rc=$?; tail -2 gpurun_out/tail4/suite.txt; exit $rc
