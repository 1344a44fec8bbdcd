#!/bin/bash
# Where the G = 10 pair kernel's wave cycles go (262144^2, unhashed): SQ
# wave-state counters in one pass, instruction counts in another, each a
# separate rocprofv3 --pmc run under its own hard limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/sq
mkdir -p $P
timeout -s KILL 60 rocprofv3 --list-avail > $P/avail.txt 2>&1
i=0
for counters in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
                "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVES SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $counters -T -d $P/pass$i -o run --output-format csv -- python3 scripts/prof_run.py 262144x262144 10 > $P/pass$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $P/pass$i.log; exit $rc; }
done
VALU_RATE_PAIR=1 timeout -k 10 60 scripts/micro/valu_rate > gpurun_out/sq/valu_rate_pair.txt 2>&1 || exit 1
# the N = 2 / 4 per-rank ring shapes at the planner's depth (pmc_launch.json rows)
CONFIGS="262144x131072:ring:10:0 262144x65536:ring:10:0 262144x32768:ring:10:1" bash scripts/gpu_pmc.sh > gpurun_out/pmc_r4ring.log 2>&1
