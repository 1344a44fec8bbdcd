# 262144^2 pass plans, same box: automatic plan vs fixed depths 7 and 8.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/plan262_ab.txt; : > $out
for r in 1 2 3; do
  for g in 0 7 8; do
    timeout -k 10 120 python3 bench.py --gpp $g --no-secondary --no-cpu > gpurun_out/p.json 2> gpurun_out/p.err || exit $?
    python3 -c "import json,sys;d=json.load(open('gpurun_out/p.json'));print('r$r gpp=$g', d['value'], d['roofline']['pass_plan'])" | tee -a $out
  done
done
