# SQ counters of library builds under ab/<name>/lib on the 262144^2 G=6 run.
#   AB="old new" bash scripts/gpu_sq_ab.sh
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=gpurun_out/sqab
mkdir -p $P
for v in ${AB:-old new}; do
  GOL_LIB_PATH=$PWD/ab/$v/lib/libgol.so timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -T -d $P/$v -o run --output-format csv -- python3 scripts/prof_run.py ${EDGE:-262144} 60 ${GPP:-0} > $P/$v.log 2>&1
  rc=$?; echo "sq $v rc=$rc"; [ $rc -eq 0 ] || { tail -20 $P/$v.log; exit $rc; }
done
python3 - <<'PY'
import csv, collections, os
for v in os.environ.get("AB", "old new").split():
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f"gpurun_out/sqab/{v}/run_counter_collection.csv")):
        if "step" in r["Kernel_Name"] and "_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    d = {k: sum(x) / len(x) for k, x in agg.items()}
    w = d["SQ_WAVE_CYCLES"]
    print(v, {k: round(x / 1e6, 1) for k, x in sorted(d.items())})
    print(v, "fractions of wave-cycles:", {k: round(d[k] / w, 3) for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA") if k in d})
PY
