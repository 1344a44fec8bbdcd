# Round 3: enqueue a sharded pass's interior launch before the RCCL exchange
# (the GPU starts it while the host is inside the RCCL group calls).  Parity
# of the ring paths first, then one N = 8 rank's shard as a 1-rank self-ring
# (scripts/band_ab.py --ring, the bench's 5 + 12 + 8 window), ab/prev (the
# exchange enqueued first) vs ab/cur, interleaved processes.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rccl.py tests/test_gpu_loopback.py \
    tests/test_gpu_group.py tests/test_gpu_hip_status.py > gpurun_out/ifirst_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/ifirst_tests.txt; [ $rc -eq 0 ] || exit $rc
for round in 1 2 3; do
  for v in prev cur; do
    GOL_LIB_PATH=$PWD/ab/$v/lib/libgol.so timeout -k 10 200 python -u scripts/band_ab.py --ring --shape 262144x32768 --rounds 3 12:0,8:0 > gpurun_out/if_ab_$v.$round.txt 2>&1
    rc=$?; [ $rc -eq 0 ] || exit $rc
    echo "$v r$round $(tail -n 1 gpurun_out/if_ab_$v.$round.txt)"
  done
done
