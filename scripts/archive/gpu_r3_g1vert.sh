# Round 3: single-generation passes with vertical workgroups (a workgroup's 4
# waves on 4 adjacent bands of one strip) vs the band-major order, interleaved
# processes; then the G = 1 parity tests.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for round in 1 2 3; do
  for v in 1 0; do
    GOL_G1_VERTICAL=$v timeout -k 10 200 python -u scripts/band_ab.py --shape 65536x65536 --rounds 3 1:0,1:0,1:0,1:0,1:0,1:0,1:0,1:0,1:0,1:0,1:0,1:0,1:0,1:0,1:0,1:0 > gpurun_out/r3_g1v$v.65536.$round.txt 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/r3_g1v$v.65536.$round.txt; exit $rc; }
    echo "v=$v 65536 r$round: $(tail -1 gpurun_out/r3_g1v$v.65536.$round.txt)"
    GOL_G1_VERTICAL=$v timeout -k 10 200 python -u scripts/band_ab.py --rounds 2 1:0,1:0,1:0,1:0 > gpurun_out/r3_g1v$v.262144.$round.txt 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/r3_g1v$v.262144.$round.txt; exit $rc; }
    echo "v=$v 262144 r$round: $(tail -1 gpurun_out/r3_g1v$v.262144.$round.txt)"
  done
done
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "unhashed_single or gpp1 or 1- or words_per_lane or snapshot or replay or rccl or group" > gpurun_out/r3_g1v_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3_g1v_tests.log; exit $rc
