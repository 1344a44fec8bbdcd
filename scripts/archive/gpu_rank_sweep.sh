cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
BANDS=0,128,160,180,200,216,240,256,320,400 TAILS=";0,0;1,3;1,2;2,3" GPPS=6,8 ROUNDS=2 timeout -k 10 300 python scripts/rank_sweep.py 262144x32768 --ring > gpurun_out/r2_rank_sweep_ring.log 2>&1
rc=$?; echo "ring rc=$rc"; [ $rc -eq 0 ] || { tail gpurun_out/r2_rank_sweep_ring.log; exit $rc; }
sort -t= -k8 -n gpurun_out/r2_rank_sweep_ring.log | head -3
BANDS=0,180,216,256,320 TAILS=";0,0;1,3" GPPS=6,8 ROUNDS=2 timeout -k 10 300 python scripts/rank_sweep.py 65536x65536 > gpurun_out/r2_rank_sweep_65536.log 2>&1
rc=$?; echo "65536 rc=$rc"; exit $rc
