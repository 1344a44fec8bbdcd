# Round 3: XCD chunk (consecutive blocks kept on one XCD) for the single-
# generation band paths: with 6-row bands the 65536^2 pass reads 1.10 planes
# and 262144^2 1.35 (PMC): band seams that cross XCDs are fetched twice.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for round in 1 2; do
  for c in 8 16 32 64; do
    for shape in 65536x65536:256 262144x262144:32; do
      IFS=: read s n <<< "$shape"
      GOL_XCD_CHUNK=$c timeout -k 10 200 python -u scripts/g1_band_path.py --shape $s --gens $n --rounds 2 6:4 \
          > gpurun_out/g1xcd_$c.$s.$round.txt 2>&1
      rc=$?; [ $rc -eq 0 ] || exit $rc
      echo "chunk=$c $s r$round $(tail -n 1 gpurun_out/g1xcd_$c.$s.$round.txt)"
    done
  done
done
