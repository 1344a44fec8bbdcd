# Round 3: (1) refresh the PMC keys of the single-generation passes (6-row
# band paths) and (2) rows prefetched ahead in the horizontal-first kernel
# (GOL_HG_PF): at 3 waves per SIMD a CU holds ~18 KB of row loads in flight
# with 2 rows ahead, about what 2.4 TB/s at ~2 us of loaded latency needs.
# Same-box A/B of the bench (no CPU / ring legs), interleaved: pf2 (default)
# vs pf3 vs pf4.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
CONFIGS="65536x65536:N1:1:0 262144x262144:N1:1:0" bash scripts/gpu_pmc.sh > gpurun_out/pmc_r3d.log 2>&1
rc=$?; tail -2 gpurun_out/pmc_r3d.log; [ $rc -eq 0 ] || exit $rc
AB="pf2 pf3 pf4" ROUNDS=3 bash scripts/gpu_ab_bench.sh > gpurun_out/r3_pf_ab.txt 2>&1
rc=$?; cat gpurun_out/r3_pf_ab.txt; exit $rc
