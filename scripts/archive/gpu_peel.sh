# Pipeline-fill peel + band tail split: GPU tests, same-box A/B against the
# previous library (ab/base, scripts/ab_build.sh base <rev>), the tail sweep,
# and one PMC pass for the effective clock / VALU issue of the bench kernel.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/peel
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for v in base new; do
    lib=$PWD/akka-game-of-life_amd/lib/libgol.so; [ $v = base ] && lib=$PWD/ab/base/lib/libgol.so
    GOL_LIB_PATH=$lib VECS=0 GPPS=6 BANDS=0 HASH=0 ROUNDS=2 \
      timeout -k 10 200 python scripts/tune.py 262144 65536 262144x32768 > $O/ab_$v.$round.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "ab $v rc=$rc"; tail -5 $O/ab_$v.$round.log; exit $rc; }
    sed "s/^/$v r$round /" $O/ab_$v.$round.log | cut -c1-120
  done
done
timeout -k 10 300 python scripts/tail_sweep.py > $O/tail_sweep.log 2>&1
rc=$?; cat $O/tail_sweep.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  -T -d $O/pmc_clk -o run --output-format csv -- python3 scripts/prof_run.py 262144 60 0 > $O/pmc_clk.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -2 $O/pmc_clk.log
exit $rc
