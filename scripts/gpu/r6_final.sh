#!/bin/bash
# Round 6 final build on one box: the GPU suite, smoke(), rocprofv3
# kernel-trace/stats of the driver's bench command (the per-launch PMC table
# is a separate call, see below), the driver's command and the default bench unprofiled, and the free
# space of the directories the N > 1 fault drill may use.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
rm -rf gpurun_out/final6 gpurun_out/prof gpurun_out/pmc; mkdir -p gpurun_out/final6 gpurun_out/prof
df -h /tmp /dev/shm > gpurun_out/final6/df.txt 2>&1
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/final6/suite.txt 2>&1 || { tail -30 gpurun_out/final6/suite.txt; exit 1; }
tail -3 gpurun_out/final6/suite.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final6/smoke.txt 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/bench_trace -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof/bench_under_rocprof.json 2> gpurun_out/prof/bench_under_rocprof.err
rc=$?; echo "rocprof trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
# the PMC passes run as their own call (gpurun's 20-minute limit):
#   CONFIGS="262144x262144:N1:10:0 262144x262144:N1:10:1 65536x65536:N1:10:0 65536x65536:N1:7:0 65536x65536:N1:1:0 262144x32768:ring:10:0" bash scripts/gpu_pmc.sh
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > gpurun_out/prof/bench_default.json 2> gpurun_out/prof/bench_default.err
rc=$?; echo "bench default rc=$rc"
python3 -c "import json; d=json.load(open('gpurun_out/prof/bench.json')); print(d['value'], d['roofline']['frac'], d['with_state_hash']['value'], d['secondary']['value'], d['parity_ok'])"
exit $rc
