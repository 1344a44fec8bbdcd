# GPU tests on the in-tree build, then same-box A/B of the XCD chunk of the
# step kernels' block order (GOL_XCD_CHUNK; 1 = plain dispatch order),
# interleaved processes, scripts/tune.py kernel time per generation.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2 3; do
  for c in ${CHUNKS:-1 4 8 16}; do
    GOL_XCD_CHUNK=$c VECS=${VECS:-2} GPPS=${GPPS:-6} BANDS=0 HASH=0 ROUNDS=2 \
      timeout -k 10 200 python scripts/tune.py ${SHAPES:-262144 65536 262144x32768} > gpurun_out/xcd_$c.$round.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "chunk $c rc=$rc"; tail -5 gpurun_out/xcd_$c.$round.log; exit $rc; }
    sed "s/^/chunk=$c r$round /" gpurun_out/xcd_$c.$round.log | cut -c1-150
  done
done
