#!/bin/bash
# Round 6: XCD chunk (GOL_XCD_CHUNK, read once per process) at G = 10 on the
# final band schedule, scored per probed GHz (scripts/band_scan.py).
set -o pipefail
mkdir -p gpurun_out/xcd
for r in 1 2; do
  for c in 1 4 8 16 32; do
    GOL_XCD_CHUNK=$c timeout -k 10 120 python -u scripts/band_scan.py 262144 10 30 '1,4' > gpurun_out/xcd/262144_c${c}_r$r.txt 2>&1 || exit 1
    GOL_XCD_CHUNK=$c timeout -k 10 120 python -u scripts/band_scan.py 65536 10 300 '1,6' > gpurun_out/xcd/65536_c${c}_r$r.txt 2>&1 || exit 1
  done
done
for f in gpurun_out/xcd/*.txt; do echo "$(basename $f) $(grep 'tail=     -' $f | tail -1)"; done
