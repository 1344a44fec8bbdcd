# Round 2: the redefined state hash (one v_mad_u64_u32 per word-generation,
# LDS sums in the horizontal-first kernel): GPU parity, hashed depth sweeps of
# the new build, the unforced G = 8 variant (ab/mw1) and the old hash
# (ab/oldhash), then the bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r2_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
HASH=1 ROUNDS=2 timeout -k 10 200 python scripts/depth_sweep.py 262144 65536 262144x32768 > gpurun_out/r2_sweep_hash_new.log 2>&1
rc=$?; echo "sweep new rc=$rc"; cat gpurun_out/r2_sweep_hash_new.log; [ $rc -eq 0 ] || exit $rc
HASH=0 ROUNDS=2 timeout -k 10 200 python scripts/depth_sweep.py 262144 65536 > gpurun_out/r2_sweep_nohash.log 2>&1
rc=$?; echo "sweep nohash rc=$rc"; cat gpurun_out/r2_sweep_nohash.log; [ $rc -eq 0 ] || exit $rc
GOL_LIB_PATH=$PWD/ab/mw1/lib/libgol.so HASH=1 ROUNDS=2 timeout -k 10 200 python scripts/depth_sweep.py 262144 65536 > gpurun_out/r2_sweep_hash_mw1.log 2>&1
rc=$?; echo "sweep mw1 rc=$rc"; cat gpurun_out/r2_sweep_hash_mw1.log; [ $rc -eq 0 ] || exit $rc
GOL_LIB_PATH=$PWD/ab/oldhash/lib/libgol.so HASH=1 ROUNDS=2 timeout -k 10 200 python scripts/depth_sweep.py 262144 65536 > gpurun_out/r2_sweep_hash_old.log 2>&1
rc=$?; echo "sweep old rc=$rc"; cat gpurun_out/r2_sweep_hash_old.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 5 > gpurun_out/r2_bench.json 2> gpurun_out/r2_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r2_bench.json; exit $rc
