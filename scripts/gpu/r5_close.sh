#!/bin/bash
# Round 5 closing check on the final tree: the GPU suite, smoke(), and the
# driver's bench command (no kernel changed since r5_final.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/close
timeout -k 10 900 python -u -m pytest -x -q --timeout 500 --timeout-method thread -m gpu tests > gpurun_out/close/suite.txt 2>&1 || { tail -30 gpurun_out/close/suite.txt; exit 1; }
tail -3 gpurun_out/close/suite.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/close/smoke.txt 2>&1 || exit 1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/close/bench.json 2> gpurun_out/close/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.load(open('gpurun_out/close/bench.json')); print(d['value'], d['roofline']['frac'], d['with_state_hash']['value'], d['secondary']['value'], d['parity_ok'])"
