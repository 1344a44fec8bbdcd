# Per-launch PMC table for bench.py's roofline (scripts/pmc_launch.py ->
# profiles/pmc_launch.json): for every (shape, mode, pass depth, hash) the
# bench can time, three separate rocprofv3 --pmc passes over
# scripts/prof_run.py -- FETCH_SIZE; WRITE_SIZE; GRBM_GUI_ACTIVE + SQ_INSTS_VALU
# + SQ_WAVES + SQ_BUSY_CYCLES (clock and VALU issue).  One counter block set
# per pass, each pass under its own hard time limit.
#   CONFIGS="262144x262144:N1:8:0 ..." bash scripts/gpu_pmc.sh
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=gpurun_out/pmc
mkdir -p $P
CONFIGS=${CONFIGS:-"262144x262144:N1:6:0 262144x262144:N1:8:0 262144x262144:N1:7:1 262144x262144:N1:6:1 262144x262144:N1:1:0 65536x65536:N1:6:0 65536x65536:N1:8:0 65536x65536:N1:6:1 65536x65536:N1:1:0 262144x32768:N1:8:0 262144x32768:ring:8:0 262144x32768:ring:6:0 262144x65536:ring:8:0 262144x65536:ring:6:0 262144x131072:ring:8:0 262144x131072:ring:6:0"}
for cfg in $CONFIGS; do
  IFS=: read shape mode G h <<< "$cfg"
  args="$shape $G"
  [ "$h" = 1 ] && args="$args --hash"
  [ "$mode" = ring ] && args="$args --ring"
  key=${shape}_${mode}_G${G}_h${h}
  for pass in fetch write clock; do
    case $pass in
      fetch) counters="FETCH_SIZE";;
      write) counters="WRITE_SIZE";;
      clock) counters="GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES";;
    esac
    timeout -s KILL 90 rocprofv3 --pmc $counters -T -d $P/${key}__$pass -o run --output-format csv -- python3 scripts/prof_run.py $args > $P/${key}__$pass.log 2>&1
    rc=$?; echo "pmc $key $pass rc=$rc"
    [ $rc -eq 0 ] || { tail -5 $P/${key}__$pass.log; exit $rc; }
  done
done
python3 scripts/pmc_launch.py $P
