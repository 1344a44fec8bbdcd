# Profiling round: rocprofv3 kernel-trace/stats of the bench command itself,
# an unprofiled bench run, and separate PMC passes (FETCH_SIZE, WRITE_SIZE)
# for HBM traffic at G = 6 (auto) and G = 1, and one pass of clock / VALU-issue
# counters (scripts/pmc_clock.py).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=gpurun_out/prof
mkdir -p $P
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $P/bench_trace -o bench --output-format csv -- python3 bench.py --steps 60 --warmup 6 --cpu-seconds 10 > $P/bench_under_rocprof.json 2> $P/bench_under_rocprof.err
rc=$?; echo "rocprof bench rc=$rc"; tail -2 $P/bench_under_rocprof.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --steps 60 --warmup 6 --cpu-seconds 10 > $P/bench.json 2> $P/bench.err
rc=$?; echo "bench rc=$rc"; cat $P/bench.json
[ $rc -eq 0 ] || exit $rc
for edge in 262144 65536; do
  for g in 0 1; do
    for c in FETCH_SIZE WRITE_SIZE; do
      gens=60; [ $edge = 65536 ] && [ $g = 0 ] && gens=102  # bench.py's timed generations
      timeout -k 10 300 rocprofv3 --pmc $c -T -d $P/pmc_${c}_${edge}_g$g -o run --output-format csv -- python3 scripts/prof_run.py $edge $gens $g > $P/pmc_${c}_${edge}_g$g.log 2>&1
      rc=$?; echo "pmc $c $edge g$g rc=$rc"
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
for edge in 262144 65536; do
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    -T -d $P/pmc_clock_$edge -o run --output-format csv -- python3 scripts/prof_run.py $edge 60 6 > $P/pmc_clock_$edge.log 2>&1
  rc=$?; echo "pmc clock $edge rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
find $P -name '*.csv' | sort
