# Round 3: band height per pass depth on the driver's window (262144^2 fresh
# board, 5 + 12 + 8 generations) and on the N = 8 per-rank shape.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export GOL_TAIL=1.0,3
timeout -k 10 300 python -u scripts/band_ab.py --rounds 5 12:0,8:0 12:576,8:384 12:768,8:512 12:1024,8:768 \
    12:768,8:256 10:0,10:0 10:768,10:768 > gpurun_out/r3_band_262144.txt 2>&1
rc=$?; tail -9 gpurun_out/r3_band_262144.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/band_ab.py --shape 262144x32768 --rounds 5 12:0,8:0 12:576,8:384 \
    12:768,8:512 12:384,8:384 > gpurun_out/r3_band_32768.txt 2>&1
rc=$?; tail -6 gpurun_out/r3_band_32768.txt; exit $rc
