#!/usr/bin/env python3
"""Band height x tail split x pass depth on one shape (the N = 8 per-rank
shard 262144 x 32768 by default), unsharded or as a 1-rank RCCL self-ring:
kernel ms per generation (HIP events on the dominant launch) and wall ms per
generation, reseeded board per measurement, min of ROUNDS interleaved rounds.

    python scripts/rank_sweep.py [WxH] [--ring]
    env: GPPS=6,8  BANDS=0,160,216  TAILS=",0,0;1,3"  ROUNDS=2  GENS=24
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife import _native as N  # noqa: E402
from gameoflife.engine import GolEngine  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    W, H = (int(v) for v in (args[0] if args else "262144x32768").split("x"))
    ring = "--ring" in sys.argv
    gpps = [int(g) for g in os.environ.get("GPPS", "6,8").split(",")]
    bands = [int(b) for b in os.environ.get("BANDS", "0,160,216").split(",")]
    tails = os.environ.get("TAILS", ";0,0;1,3").split(";")
    rounds = int(os.environ.get("ROUNDS", "2"))
    gens = int(os.environ.get("GENS", "24"))
    res = {}
    with GolEngine(W, H) as e:
        if ring:
            e.comm_init(N.unique_id(), 0, 1)
        for _ in range(rounds):
            for G in gpps:
                for b in bands:
                    for t in tails:
                        if t:
                            os.environ["GOL_TAIL"] = t
                        else:
                            os.environ.pop("GOL_TAIL", None)
                        e.set_tuning(band_rows=b, gens_per_pass=G)
                        e.seed(0x5EED)
                        e.step(G)
                        e.sync()
                        e.profile(True)
                        e.profile_reset()
                        t0 = time.perf_counter()
                        e.step(gens)
                        e.sync()
                        wall = (time.perf_counter() - t0) / gens * 1e3
                        ms, n, g = e.profile_read()
                        e.profile(False)
                        res.setdefault((G, b, t), []).append((ms / g, wall))
    for (G, b, t), v in res.items():
        k = min(x[0] for x in v)
        w = min(x[1] for x in v)
        print(f"shape={W}x{H} ring={int(ring)} G={G} band={b:4d} tail={t or 'auto':5s} kernel_ms/gen={k:.4f} "
              f"wall_ms/gen={w:.4f} GCUPS(wall)={W * H / w / 1e6:9.1f}", flush=True)


if __name__ == "__main__":
    main()
