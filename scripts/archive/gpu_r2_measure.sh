# Round 2 measurement set: per-launch PMC table (scripts/gpu_pmc.sh), then the
# bench with no flags (its roofline reads profiles/pmc_launch.json, which is
# summarised on the CPU side afterwards).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/gpu_pmc.sh > gpurun_out/r2_pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -25 gpurun_out/r2_pmc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r2_bench_default.json 2> gpurun_out/r2_bench_default.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r2_bench_default.json; tail -3 gpurun_out/r2_bench_default.err; exit $rc
