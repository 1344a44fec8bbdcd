# Tail-split sweep with a reseeded board per measurement (scripts/tail_sweep.py).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tail
TAILS="0,0;1,2;1,3;2,2;2,3;3,3" BANDS=0 ROUNDS=4 timeout -k 10 400 python scripts/tail_sweep.py 262144x32768 65536 262144x65536 262144x131072 > gpurun_out/tail/tail_sweep.log 2>&1
rc=$?; cat gpurun_out/tail/tail_sweep.log; exit $rc
