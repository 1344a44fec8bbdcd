# Pass-mix A/B for the planner's cost table (scripts/plan_mix_ab.py): the
# driver's 20-generation window at 262144^2 and the N = 8 per-rank shape,
# unhashed and hashed.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=gpurun_out/plan_ab.log
: > $L
timeout -k 10 200 python scripts/plan_mix_ab.py --rounds 4 6,6,8 10,10 8,12 12,8 9,11 11,9 >> $L 2>&1 || exit $?
timeout -k 10 200 python scripts/plan_mix_ab.py --rounds 4 --hash 6,7,7 6,6,8 10,10 6,6,6,2 9,11 >> $L 2>&1 || exit $?
timeout -k 10 200 python scripts/plan_mix_ab.py --shape 262144x32768 --rounds 4 6,6,8 10,10 8,12 9,11 12,8 >> $L 2>&1 || exit $?
timeout -k 10 200 python scripts/plan_mix_ab.py --rounds 3 8,8,8,8,8,8,8,4 10,10,10,10,10,10 12,12,12,12,12 11,11,11,11,11,5 >> $L 2>&1 || exit $?
grep best $L
