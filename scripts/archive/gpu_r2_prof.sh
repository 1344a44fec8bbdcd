# Round-2 profile of the driver's bench command: rocprofv3 --kernel-trace
# --stats of `bench.py --steps 20 --warmup 5` and the same command unprofiled
# (scripts/prof_summary.py turns both into profiles/<tag>_*).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=gpurun_out/prof
mkdir -p $P
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/bench_trace -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 > $P/bench_under_rocprof.json 2> $P/bench_under_rocprof.err
rc=$?; echo "rocprof bench rc=$rc"; tail -c 400 $P/bench_under_rocprof.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $P/bench.json 2> $P/bench.err
rc=$?; echo "bench rc=$rc"; cat $P/bench.json
exit $rc
