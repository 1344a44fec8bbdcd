# GPU tests, then the bench (unprofiled) and the same bench command under
# rocprofv3 --kernel-trace --stats (per-kernel durations for profiles/).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/bench
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python3 bench.py > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err
rc=$?; echo "rocprof rc=$rc"; exit $rc
