#!/bin/bash
# Round 6, VERDICT r05 item 1 (one measurement): the step kernels with delta
# row pointers (gol_stencil.h RowAddr: no per-row kernarg s_load, so no
# lgkmcnt(0) drain between the hashed kernel's LDS adds) against round 5's
# build (lib_ab/base/libgol.so, built from the round-5 head), the driver's
# command, same box, interleaved.  Parity first: the GPU parity and full-size
# suites on the new build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
rm -rf gpurun_out/rowaddr; mkdir -p gpurun_out/rowaddr
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py > gpurun_out/rowaddr/parity.txt 2>&1 || { tail -40 gpurun_out/rowaddr/parity.txt; exit 1; }
tail -2 gpurun_out/rowaddr/parity.txt
B="python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu"
for r in 1 2 3; do
  GOL_LIB_PATH=$PWD/akka-game-of-life_amd/lib_ab/base/libgol.so timeout -k 10 200 $B > gpurun_out/rowaddr/base_$r.json 2>gpurun_out/rowaddr/base_$r.err || exit 1
  timeout -k 10 200 $B > gpurun_out/rowaddr/new_$r.json 2>gpurun_out/rowaddr/new_$r.err || exit 1
  echo "round $r done"
done
python3 - <<'PY'
import json, glob
for k in ("base", "new"):
    for f in sorted(glob.glob(f"gpurun_out/rowaddr/{k}_*.json")):
        d = json.load(open(f))
        h = d["with_state_hash"]
        print(k, d["value"], d["roofline"]["avg_launch_ms"], d["roofline"]["held_clock"].get("ghz"),
              h["value"], h["roofline"]["avg_launch_ms"], d["secondary"]["value"],
              d["secondary"]["single_generation_passes"]["value"], d["parity_ok"])
PY
