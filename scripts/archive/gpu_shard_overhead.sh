cd $GRAFT_REPO_ROOT
for v in base edge base edge; do
  GOL_LIB_PATH=$PWD/ab/$v/lib/libgol.so timeout -k 10 200 python scripts/shard_overhead.py 262144 65536 2 48 > gpurun_out/so_$v.log 2>&1 || { cat gpurun_out/so_$v.log; exit 1; }
  echo "$v $(cat gpurun_out/so_$v.log)"
  GOL_LIB_PATH=$PWD/ab/$v/lib/libgol.so timeout -k 10 300 python scripts/shard_overhead.py 262144 262144 8 24 > gpurun_out/so8_$v.log 2>&1 || { cat gpurun_out/so8_$v.log; exit 1; }
  echo "$v $(cat gpurun_out/so8_$v.log)"
done
