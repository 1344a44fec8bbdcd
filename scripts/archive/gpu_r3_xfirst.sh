# Round 3: the sharded pass's schedule on one N = 8 rank's shard (262144 x 32768,
# 1-rank self-ring): overlap (interior || exchange, then boundary rows) vs
# exchange-first (exchange, then one launch over the whole shard), and the
# same shard without a ring.  Parity of the exchange-first schedule first.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
GOL_EXCHANGE=first timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_loopback.py tests/test_gpu_rccl.py > gpurun_out/xfirst_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/xfirst_tests.txt; [ $rc -eq 0 ] || exit $rc
for v in first overlap; do
  GOL_EXCHANGE=$v timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/xf_$v -o rank --output-format csv -- python3 scripts/rank_window_trace.py > gpurun_out/xf_trace_$v.txt 2>&1
  rc=$?; grep window gpurun_out/xf_trace_$v.txt; [ $rc -eq 0 ] || exit $rc
done
for round in 1 2 3; do
  for v in first overlap; do
    GOL_EXCHANGE=$v timeout -k 10 200 python -u scripts/band_ab.py --ring --shape 262144x32768 --rounds 3 12:0,8:0 > gpurun_out/xf_ab_$v.$round.txt 2>&1
    rc=$?; [ $rc -eq 0 ] || exit $rc
    echo "$v r$round $(tail -n 1 gpurun_out/xf_ab_$v.$round.txt)"
  done
  timeout -k 10 200 python -u scripts/band_ab.py --shape 262144x32768 --rounds 3 12:0,8:0 > gpurun_out/xf_ab_noring.$round.txt 2>&1
  rc=$?; [ $rc -eq 0 ] || exit $rc
  echo "no-ring r$round $(tail -n 1 gpurun_out/xf_ab_noring.$round.txt)"
done
