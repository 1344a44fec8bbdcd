# Round 3: the single-generation XCD chunk rule (4 x blocks per band) --
# parity (block order, single-generation checks) and the default's rate.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_xcd_order.py tests/test_gpu_parity.py \
    -k "order or single" > gpurun_out/g1xcd2_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/g1xcd2_tests.txt; [ $rc -eq 0 ] || exit $rc
for shape in 262144x262144:32 65536x65536:256 262144x32768:256; do
  IFS=: read s n <<< "$shape"
  timeout -k 10 200 python -u scripts/g1_band_path.py --shape $s --gens $n --rounds 3 0:0 > gpurun_out/g1xcd2_$s.txt 2>&1
  rc=$?; [ $rc -eq 0 ] || exit $rc
  echo "$s $(tail -n 1 gpurun_out/g1xcd2_$s.txt)"
done
