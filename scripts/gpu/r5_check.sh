#!/bin/bash
# Round 5: the GPU suite, smoke() and the driver's bench command on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r5_suite.txt 2>&1 || { tail -30 gpurun_out/r5_suite.txt; exit 1; }
tail -3 gpurun_out/r5_suite.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_smoke.txt 2>&1 || exit 1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5_bench.json 2> gpurun_out/r5_bench.err
rc=$?
python3 -c "import json; d=json.load(open('gpurun_out/r5_bench.json')); print(d['value'], d['roofline']['frac'], d['with_state_hash']['value'], d['parity_ok'], d['parity_failed'])"
exit $rc
