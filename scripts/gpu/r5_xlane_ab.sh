#!/bin/bash
# Round 5, VERDICT r04 item 2 (one experiment): pair passes with the
# cross-lane words over ds_bpermute one step ahead (GOL_XLANE=lds, G = 7:
# the deepest depth at 3 waves per SIMD without spilling) against today's
# DPP build (the planner's 10 + 10, and G = 7 fixed), the driver's command,
# same box, interleaved.  Parity first: the bp kernel suite and the fault drill.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
rm -rf gpurun_out/xlane; mkdir -p gpurun_out/xlane
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_xlane.py tests/test_gpu_fault_drill.py > gpurun_out/xlane/parity.txt 2>&1 || { tail -40 gpurun_out/xlane/parity.txt; exit 1; }
tail -2 gpurun_out/xlane/parity.txt
B="python3 bench.py --steps 20 --warmup 5 --no-secondary --no-ring --no-cpu"
for r in 1 2 3; do
  timeout -k 10 200 $B > gpurun_out/xlane/dpp_plan_$r.json 2>/dev/null || exit 1
  GOL_XLANE=lds timeout -k 10 200 $B --gpp 7 > gpurun_out/xlane/lds_g7_$r.json 2>/dev/null || exit 1
  timeout -k 10 200 $B --gpp 7 > gpurun_out/xlane/dpp_g7_$r.json 2>/dev/null || exit 1
  GOL_XLANE=lds timeout -k 10 200 $B --gpp 8 > gpurun_out/xlane/lds_g8_$r.json 2>/dev/null || exit 1
  echo "round $r done"
done
python3 - <<'PY'
import json, glob
for k in ("dpp_plan", "lds_g7", "dpp_g7", "lds_g8"):
    vals = []
    for f in sorted(glob.glob(f"gpurun_out/xlane/{k}_*.json")):
        d = json.load(open(f))
        vals.append((d["value"], d["roofline"]["avg_launch_ms"], d["roofline"]["pass_plan"], d["roofline"]["held_clock"].get("ghz"), d["parity_ok"]))
    print(k, vals)
PY
