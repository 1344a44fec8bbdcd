# Round 3 round-end rehearsal on a fresh box: PMC refresh of the N = 2 ring
# shard keys (tall bands changed them), the GPU suite, smoke(), the default
# bench and the driver's command.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
CONFIGS="262144x131072:ring:12:0 262144x131072:ring:8:0" bash scripts/gpu_pmc.sh > gpurun_out/pmc_r3b.log 2>&1
rc=$?; tail -2 gpurun_out/pmc_r3b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_final_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r3_final_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/r3_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r3_bench_default.json 2> gpurun_out/r3_bench_default.err
rc=$?; echo "bench default rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3_bench_driver.json 2> gpurun_out/r3_bench_driver.err
rc=$?; echo "bench driver rc=$rc"; exit $rc
