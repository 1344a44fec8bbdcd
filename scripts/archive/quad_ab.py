"""Quad layout vs pair layout, same box (VERDICT r03 item 3 follow-up).

    python scripts/quad_ab.py pairs|quads [out.json]

GOL_LAYOUT=quads makes quad-capable tori quad-interleaved.  For each layout:
ms per generation of the bench's window (seed, 100 ms settle, re-seed, 5 + 20
generations) at 262144^2 for several fixed pass depths and the planner's
choice, and a digest of the row-major 65536^2 board after 200 generations
(the two layouts must agree bit for bit: gol_snapshot de-interleaves)."""
import hashlib
import json
import os
import sys
import time

mode = sys.argv[1]
if mode == "quads":
    os.environ["GOL_LAYOUT"] = "quads"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))
from gameoflife.engine import GolEngine  # noqa: E402

out = {"mode": mode, "rows": []}


def window(e, gpp, W, H, K=20, Wu=5):
    e.set_tuning(gens_per_pass=gpp)
    e.seed(0x5EED)
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) < 0.1:
        e.step(12)
        e.sync()
    e.seed(0x5EED)
    e.step(Wu)
    e.sync()
    e.profile(True)
    e.profile_reset()
    t0 = time.perf_counter()
    e.step(K)
    e.sync()
    dt = time.perf_counter() - t0
    ms, n, g = e.profile_read()
    clk = e.profile_clock()
    e.profile(False)
    return {"gpp": gpp, "plan": e.pass_plan(K), "ms_per_gen": round(dt / K * 1e3, 4),
            "gcups": round(W * H * K / dt / 1e9, 1), "kernel_ms_per_gen": round(ms / max(g, 1), 4),
            "clock_ghz": round(clk, 3)}


S = 65536
with GolEngine(S, S) as e:
    e.seed(0x5EED)
    e.step(200)
    snap = e.snapshot()
    out["digest_65536_200"] = hashlib.sha1(snap.tobytes()).hexdigest()
    out["occupancy"] = {g: e.occupancy(g) for g in (6, 7, 8, 12)}
    for gpp in (0, 8):
        out["rows"].append(dict(board=S, **window(e, gpp, S, S, K=256, Wu=12)))
W = 262144
with GolEngine(W, W) as e:
    for gpp in ([0, 6, 7, 8, 12] if mode == "pairs" else [0, 6, 7, 8, 10, 12]):
        out["rows"].append(dict(board=W, **window(e, gpp, W, W)))
        print(json.dumps(out["rows"][-1]), flush=True)
print(json.dumps(out))
if len(sys.argv) > 2:
    with open(sys.argv[2], "w") as f:
        json.dump(out, f, indent=1)
