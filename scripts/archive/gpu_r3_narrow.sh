# Round 3: 65536^2 depth x band (does a single round of 384-row tiles let the
# deep passes win on the narrow board?).  Run 1: fixed bands without the tail
# split; run 2: GOL_TAIL=1.0,3 keeps the default tail split on fixed bands.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
GOL_TAIL=1.0,3 timeout -k 10 400 python -u scripts/narrow_band_depth.py --rounds 3 8:0 8:256 8:320 10:320 10:384 12:320 12:384 12:448 \
    > gpurun_out/r3_narrow_band_depth_tail.txt 2>&1
rc=$?; tail -10 gpurun_out/r3_narrow_band_depth_tail.txt; exit $rc
