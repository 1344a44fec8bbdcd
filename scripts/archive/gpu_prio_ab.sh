# Same-box A/B: halo-exchange and boundary-row streams at the highest
# priority (default) vs plain priorities (GOL_STREAM_PRIO=0), on the per-rank
# self-ring shapes of N = 8 / 4 and the whole board, interleaved processes.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/prio_ab.log
for r in 1 2 3; do
  for v in hi plain; do
    if [ $v = plain ]; then P=0; else P=1; fi
    for shape in 262144x32768 262144x65536; do
      GOL_STREAM_PRIO=$P GPPS=12,8 BANDS=0 TAILS=";" ROUNDS=1 GENS=48 timeout -k 10 120 python scripts/rank_sweep.py $shape --ring 2>&1 | grep shape= | sed "s/^/$v r$r /" >> gpurun_out/prio_ab.log || exit 1
    done
  done
done
cat gpurun_out/prio_ab.log
