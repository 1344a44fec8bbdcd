# Same-box A/B of library builds (ab/<name>, scripts/ab_build.sh) on the
# driver's bench command (--steps 20 --warmup 5, no CPU baseline / ring runs),
# interleaved rounds.   AB="old new" ROUNDS=3 bash scripts/gpu_ab_bench.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-3}); do
  for v in ${AB:-old new}; do
    GOL_LIB_PATH=$PWD/ab/$v/lib/libgol.so timeout -k 10 200 python bench.py --no-cpu --no-ring --steps ${STEPS:-20} --warmup ${WARMUP:-5} > gpurun_out/ab_bench_$v.$r.json 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || { echo "ab $v rc=$rc"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_bench_$v.$r.json')); print('$v r$r', 'value', d['value'], 'hashed', d.get('with_state_hash',{}).get('value'), 'secondary', d['secondary']['value'], 'single', d['secondary']['single_generation_passes']['value'])"
  done
done
