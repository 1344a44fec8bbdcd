# Round 3: split-stage kernel (variant 3: one tile per 2-wave workgroup, stages
# 1..G/2 in the producer wave, G/2+1..G in the consumer, stage-G/2 rows through
# LDS).  Parity first (every unhashed depth, bands, full size, group, RCCL
# self-ring, loopback ring), then a same-box A/B of the driver's bench command
# against GOL_SPLIT_STAGES=0 (the 3-wave horizontal-first kernel), interleaved.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_unhashed_passes.py tests/test_gpu_fullsize.py \
    -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r3_split_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3_split_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in 0 1; do
    GOL_SPLIT_STAGES=$v timeout -k 10 200 python bench.py --no-cpu --no-ring --steps 20 --warmup 5 > gpurun_out/ab_split_$v.$r.json 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || { echo "ab $v rc=$rc"; exit $rc; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_split_$v.$r.json')); r=d['roofline']; print('split=$v r$r', 'value', d['value'], 'clock', r['held_clock'].get('ghz'), 'match', d['parity']['match'], 'hashed', d['with_state_hash']['value'], 'secondary', d['secondary']['value'])"
  done
done
