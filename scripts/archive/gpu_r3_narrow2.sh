# Round 3: 65536^2 at G = 8, bands below 256 (with the tail split); 8:256 first
# and last to show the drift of a board that thins out during the run.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
GOL_TAIL=1.0,3 timeout -k 10 400 python -u scripts/narrow_band_depth.py --rounds 3 8:256 8:192 8:128 8:224 8:160 8:256 \
    > gpurun_out/r3_narrow_band2.txt 2>&1
rc=$?; tail -8 gpurun_out/r3_narrow_band2.txt; exit $rc
