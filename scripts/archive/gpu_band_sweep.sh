# Band height x tail split at G = 6 and 8 on the bench's shapes (GPU busy,
# reseeded board per measurement): the table behind pick_band / tail_split.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for shape in 262144x262144 65536x65536 262144x32768 262144x65536 262144x131072; do
  BANDS=0,216,256,320,400,512 TAILS=";0,0;1,3;1,2;2,3" GPPS=6,8 ROUNDS=2 GENS=24 timeout -k 10 300 python scripts/rank_sweep.py $shape > gpurun_out/r2_band_$shape.log 2>&1
  rc=$?; echo "$shape rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/r2_band_$shape.log; exit $rc; }
done
for v in cur hreg cur hreg; do
  GOL_LIB_PATH=$PWD/ab/$v/lib/libgol.so HASH=1 ROUNDS=1 timeout -k 10 200 python scripts/depth_sweep.py 262144 65536 >> gpurun_out/r2_hash_lds_ab_$v.log 2>&1
  rc=$?; echo "hash ab $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
