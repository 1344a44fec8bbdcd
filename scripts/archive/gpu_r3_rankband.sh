# Round 3: band heights of one N = 8 rank's shard (262144 x 32768 as a 1-rank
# self-ring: the interior launch is 32744 rows at G = 12) -- one round of
# 728-row bands (45 bands x 67 strips = 3015 of 3072 resident waves), two of
# 364, three of 243, the automatic 256 -- with and without the tail split.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFG="12:0,8:0 12:728,8:546 12:364,8:364 12:243,8:273 12:728,8:728"
GOL_TAIL=1.0,3 timeout -k 10 300 python -u scripts/band_ab.py --ring --shape 262144x32768 --rounds 5 $CFG > gpurun_out/r3_rankband_tail.txt 2>&1
rc=$?; tail -6 gpurun_out/r3_rankband_tail.txt; [ $rc -eq 0 ] || exit $rc
GOL_TAIL=0,0 timeout -k 10 300 python -u scripts/band_ab.py --ring --shape 262144x32768 --rounds 5 $CFG > gpurun_out/r3_rankband_notail.txt 2>&1
rc=$?; tail -6 gpurun_out/r3_rankband_notail.txt; exit $rc
