#!/bin/bash
# Round 6: the stream-copy peak (scripts/micro/copy_bw, grid-stride and
# one-shot tile variants), rocprofv3 --kernel-trace --stats of the driver's
# bench command, the same command unprofiled, and the default 60-generation
# bench (profiles/r06_*).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/prof
rm -rf $P gpurun_out/r6prof; mkdir -p $P gpurun_out/r6prof
timeout -k 10 120 ./scripts/micro/copy_bw > gpurun_out/r6prof/copy_bw.txt 2>&1 || { cat gpurun_out/r6prof/copy_bw.txt; exit 1; }
tail -1 gpurun_out/r6prof/copy_bw.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/bench_trace -o bench --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $P/bench_under_rocprof.json 2> $P/bench_under_rocprof.err
rc=$?; echo "rocprof trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $P/bench.json 2> $P/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > $P/bench_default.json 2> $P/bench_default.err
rc=$?; echo "bench default rc=$rc"
python3 -c "
import json
for f in ('bench_under_rocprof', 'bench', 'bench_default'):
    d = json.load(open('$P/' + f + '.json')); r = d['roofline']
    print(f, d['value'], r['frac'], r.get('frac_guide_issue'), r['avg_launch_ms'], d['with_state_hash']['value'], d['secondary']['value'], d['parity_ok'])
"
exit $rc
