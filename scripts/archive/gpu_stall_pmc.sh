# Where do the step kernel's wave-cycles go?  One PMC pass per config:
# SQ_WAVE_CYCLES = SQ_WAIT_ANY (parked on s_waitcnt) + SQ_WAIT_INST_ANY
# (issue stall) + SQ_ACTIVE_INST_ANY (MI355X_MICROARCH.md "rocprofv3 PMC slots").
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=gpurun_out/stall
mkdir -p $P
IFS=";" read -ra CFG_LIST <<< "${CFGS:-262144x262144 8;262144x262144 6;262144x262144 6 --hash;65536x65536 8;262144x32768 8}"
for cfg in "${CFG_LIST[@]}"; do
  key=$(echo $cfg | tr ' ' '_' | tr -d '-')
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -T -d $P/$key -o run --output-format csv -- python3 scripts/prof_run.py $cfg > $P/$key.log 2>&1
  rc=$?; echo "$key rc=$rc"; [ $rc -eq 0 ] || { tail -5 $P/$key.log; exit $rc; }
done
