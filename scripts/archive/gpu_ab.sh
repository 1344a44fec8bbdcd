# Same-box A/B of library builds under ab/<name>/lib (scripts/ab_build.sh):
# interleaved processes A B A B ..., each a short scripts/tune.py sweep.
#   AB="old new" SHAPES="262144 65536" GPPS=6 bash scripts/gpu_ab.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for round in 1 2 3; do
  for v in ${AB:-old new}; do
    GOL_LIB_PATH=$PWD/ab/$v/lib/libgol.so VECS=${VECS:-2} GPPS=${GPPS:-6} BANDS=${BANDS:-0} HASH=0 ROUNDS=2 \
      timeout -k 10 200 python scripts/tune.py ${SHAPES:-262144 65536} > gpurun_out/ab_$v.$round.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "ab $v rc=$rc"; tail -5 gpurun_out/ab_$v.$round.log; exit $rc; }
    sed "s/^/$v r$round /" gpurun_out/ab_$v.$round.log | cut -c1-150
  done
done
