# Same-box A/B of pass depth on the driver's bench command with the deep
# build (ab/deep: up to 12 generations per pass): the planner's plan vs fixed
# 10 / 12 generations per pass, interleaved rounds.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export GOL_LIB_PATH=$PWD/ab/deep/lib/libgol.so
for r in 1 2 3; do
  for g in 0 10 12; do
    timeout -k 10 200 python bench.py --no-cpu --no-ring --no-secondary --steps 20 --warmup 5 --gpp $g > gpurun_out/deep_ab_$g.$r.json 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || { echo "gpp $g rc=$rc"; exit $rc; }
    python3 -c "import json; d=json.load(open('gpurun_out/deep_ab_$g.$r.json')); h=d['with_state_hash']; print('gpp $g r$r', 'value', d['value'], d['roofline']['pass_plan'], 'hashed', h['value'], h['pass_plan'])"
  done
done
