# Round 3: unhashed G = 9..12 forced to 4 waves per SIMD (ab/w4: built with
# -DGOL_HG_MINWAVES_U=4, 5-10 dwords spilled) against the default 3-wave
# instances, interleaved processes A B A B, same fresh-board protocol.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export GOL_TAIL=1.0,3
CFG="12:0,8:0 9:0,9:0,9:0 10:0,10:0 11:0,11:0 12:0,12:0"
for round in 1 2 3; do
  for v in base w4; do
    if [ $v = base ]; then L=$PWD/akka-game-of-life_amd/lib/libgol.so; else L=$PWD/ab/w4/lib/libgol.so; fi
    GOL_LIB_PATH=$L timeout -k 10 200 python -u scripts/band_ab.py --rounds 2 $CFG > gpurun_out/r3_waves_$v.$round.txt 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 gpurun_out/r3_waves_$v.$round.txt; exit $rc; }
    echo "== $v round $round"; tail -6 gpurun_out/r3_waves_$v.$round.txt
  done
done
