cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VECS=2 GPPS=6 BANDS=0,96,128,160,192,216,240,256,320 HASH=0 ROUNDS=3 timeout -k 10 600 python scripts/tune.py 262144x32768 262144x65536 65536 > gpurun_out/n8shape.log 2>&1
echo "rc=$?"; cat gpurun_out/n8shape.log
