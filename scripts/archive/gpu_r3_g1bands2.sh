# Round 3: single-generation band heights with the straight-line band paths
# on the wide shapes (262144^2 and one N = 8 rank's shard) and 65536^2.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for shape in 262144x262144:64 262144x32768:256 65536x65536:256; do
  IFS=: read s n <<< "$shape"
  timeout -k 10 300 python -u scripts/g1_band_path.py --shape $s --gens $n --rounds 3 4:4 6:4 8:4 > gpurun_out/g1bands2_$s.txt 2>&1
  rc=$?; [ $rc -eq 0 ] || exit $rc
  echo "== $s"; tail -4 gpurun_out/g1bands2_$s.txt
done
