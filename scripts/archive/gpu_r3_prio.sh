# Round 3: does a high-priority comm / edge stream start a pass's RCCL kernel
# before the interior launch's waves fill the GPU?  Kernel traces of one
# N = 8 rank's window (self-ring), priority on and off.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 1 0; do
  GOL_STREAM_PRIO=$v timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/prio$v -o rank --output-format csv -- python3 scripts/rank_window_trace.py > gpurun_out/prio$v.txt 2>&1
  rc=$?; grep window gpurun_out/prio$v.txt; [ $rc -eq 0 ] || exit $rc
done
for round in 1 2 3; do
  for v in 1 0; do
    GOL_STREAM_PRIO=$v timeout -k 10 200 python -u scripts/band_ab.py --ring --shape 262144x32768 --rounds 3 12:0,8:0 > gpurun_out/prio_ab$v.$round.txt 2>&1
    rc=$?; [ $rc -eq 0 ] || exit $rc
    echo "prio=$v r$round $(tail -1 gpurun_out/prio_ab$v.$round.txt)"
  done
done
