# Band height at G = 12 with the default tail split (1 resident round in
# bands of a third), 4 interleaved rounds, on the bench's wide shapes.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/deep_band2.log
for shape in 262144x262144 262144x32768 262144x65536 262144x131072; do
  BANDS=0,256,320,384,448,512 TAILS="1,3" GPPS=12 ROUNDS=4 GENS=60 timeout -k 10 300 python scripts/rank_sweep.py $shape >> gpurun_out/deep_band2.log 2>&1
  rc=$?; echo "$shape rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/deep_band2.log; exit $rc; }
done
cat gpurun_out/deep_band2.log
