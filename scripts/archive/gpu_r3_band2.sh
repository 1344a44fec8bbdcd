# Round 3: the tall-band rule (pick_band) against the previous bands, hashed
# on 262144^2 and unhashed on the N = 2 shard shape; then the driver command.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export GOL_TAIL=1.0,3
timeout -k 10 300 python -u scripts/band_ab.py --hash --rounds 5 10:0,10:0 10:384,10:384 10:768,10:768 \
    > gpurun_out/r3_band_hash.txt 2>&1
rc=$?; tail -4 gpurun_out/r3_band_hash.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/band_ab.py --shape 262144x131072 --rounds 5 12:0,8:0 12:384,8:256 12:1024,8:768 \
    > gpurun_out/r3_band_131072.txt 2>&1
rc=$?; tail -4 gpurun_out/r3_band_131072.txt; [ $rc -eq 0 ] || exit $rc
unset GOL_TAIL
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r3_bench20_b.json 2> gpurun_out/r3_bench20_b.err
rc=$?; python -c "
import json; d=json.load(open('gpurun_out/r3_bench20_b.json'))
print(d['value'], d['roofline']['frac'], d['parity']['match'], d['with_state_hash']['value'], d['secondary']['value'], d['ring_schedule_n1']['per_rank_shard_driver_window']['value'])"
exit $rc
