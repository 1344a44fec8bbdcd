# Band height x tail split at the deep passes (G = 10, 12) on the bench's wide
# shapes: the table behind pick_band / tail_split for G > 8.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/deep_band.log
for shape in 262144x262144 262144x32768; do
  BANDS=0,256,320,384,512,640 TAILS=";0,0;1,3" GPPS=12,10 ROUNDS=2 GENS=60 timeout -k 10 300 python scripts/rank_sweep.py $shape >> gpurun_out/deep_band.log 2>&1
  rc=$?; echo "$shape rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/deep_band.log; exit $rc; }
done
cat gpurun_out/deep_band.log
