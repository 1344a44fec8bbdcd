# Round 3: single-generation band heights with the straight-line band paths
# (4, 6, 8 rows; the kernel holding all three paths has 77 VGPRs at 16-byte
# lanes, 6 waves/SIMD) against the build with the 4-row path only (55 VGPRs).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "single or band" > gpurun_out/g1bands_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/g1bands_tests.txt; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for v in b4only b468; do
    GOL_LIB_PATH=$PWD/ab/$v/lib/libgol.so timeout -k 10 200 python -u scripts/g1_band_path.py --rounds 2 4:4 6:4 8:4 4:2 8:2 \
        > gpurun_out/g1bands_$v.$round.txt 2>&1
    rc=$?; [ $rc -eq 0 ] || exit $rc
    echo "== $v round $round"; tail -6 gpurun_out/g1bands_$v.$round.txt
  done
done
