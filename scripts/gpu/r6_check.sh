#!/bin/bash
# Round 6: the measured stream-copy peak (scripts/micro/copy_bw, built here),
# the GPU suite on the split C ABI, smoke() and the driver's bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
rm -rf gpurun_out/r6; mkdir -p gpurun_out/r6
timeout -k 10 120 ./scripts/micro/copy_bw > gpurun_out/r6/copy_bw.txt 2>&1 || { cat gpurun_out/r6/copy_bw.txt; exit 1; }
tail -1 gpurun_out/r6/copy_bw.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r6/suite.txt 2>&1 || { tail -40 gpurun_out/r6/suite.txt; exit 1; }
tail -3 gpurun_out/r6/suite.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/smoke.txt 2>&1 || { tail -20 gpurun_out/r6/smoke.txt; exit 1; }
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6/bench.json 2> gpurun_out/r6/bench.err
rc=$?
python3 -c "import json; d=json.load(open('gpurun_out/r6/bench.json')); r=d['roofline']; print(d['value'], r['frac'], r.get('frac_guide_issue'), r.get('issue_rate'), d['with_state_hash']['value'], d['parity_ok'], d['parity_failed']); print(json.dumps(d.get('cpu_baseline'))[:1500])"
exit $rc
