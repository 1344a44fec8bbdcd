# SQ/GRBM counters for the step kernels (separate pass per counter group).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=gpurun_out/sq
mkdir -p $P
for g in 0 1; do
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -T -d $P/sq_g$g -o run --output-format csv -- python3 scripts/prof_run.py 262144 60 $g > $P/sq_g$g.log 2>&1
  rc=$?; echo "sq g$g rc=$rc"; [ $rc -eq 0 ] || { tail -20 $P/sq_g$g.log; exit $rc; }
done
python3 - <<'PY'
import csv, collections
for g in (0, 1):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f"gpurun_out/sq/sq_g{g}/run_counter_collection.csv")):
        if "step" in r["Kernel_Name"] and "_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("G" if g == 0 else "G1", {k: round(sum(v) / len(v)) for k, v in agg.items()})
PY
