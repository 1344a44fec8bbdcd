# Round 3: single-generation passes -- a straight-line path for the 4-row
# bands (six stream rows issued at once, four steps) and non-temporal loads
# of the two middle rows, which no other wave reads.  Parity first (the
# unhashed single-generation checks, full size), then the bench's 65536^2
# single-generation line: ab/base (HEAD) vs ab/b4 (band-4 path, plain loads)
# vs ab/b4nt (band-4 path + nt middle rows), interleaved.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
    tests/test_gpu_snapshot.py -k "single or unhashed or 65536 or snapshot or torus_life or band" > gpurun_out/g1b4_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/g1b4_tests.txt; [ $rc -eq 0 ] || exit $rc
AB="base b4 b4nt" ROUNDS=3 bash scripts/gpu_ab_bench.sh > gpurun_out/r3_g1b4_ab.txt 2>&1
rc=$?; cat gpurun_out/r3_g1b4_ab.txt; exit $rc
