#!/usr/bin/env python3
"""Band height x tail split at a fixed depth on one board, interleaved over
rounds, scored by kernel GCUPS per probed GHz (the held clock varies by box
and over a run; the per-GHz rate does not).

    python scripts/band_scan.py [EDGE|WxH] [G] [GENS] [TAILS] [h]
GOL_TAIL="frac,div" forces the tail split (gol_schedule.cpp tail_split);
TAILS ("f,d;B@f,d;B@-;...") scans only those, at the automatic band or at
band B (with that tail, or none); "h" times the
hashed passes.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife.engine import GolEngine  # noqa: E402


def main():
    shape = sys.argv[1] if len(sys.argv) > 1 else "65536"
    W, H = (int(x) for x in shape.split("x")) if "x" in shape else (int(shape), int(shape))
    G = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 300
    hashed = len(sys.argv) > 5 and sys.argv[5] == "h"
    cfgs = [(0, None)]
    if len(sys.argv) > 4 and sys.argv[4]:
        for t in sys.argv[4].split(";"):  # "f,d" at the automatic band, or "B@f,d" / "B@-" at a fixed one
            b, _, t = t.rpartition("@")
            cfgs.append((int(b) if b else 0, None if t == "-" else t))
    else:
        cfgs += [(0, t) for t in ("0", "0.5,3", "1,2", "1,4", "2,3")]
        cfgs += [(b, None) for b in (192, 256, 320, 384, 448, 512, 768)]
        cfgs += [(b, "1,3") for b in (320, 384, 512, 768)]
    res = {c: [] for c in cfgs}
    with GolEngine(W, H) as e:
        e.seed(0x5EED)
        e.step(20)
        e.sync()
        for rnd in range(3):
            for band, tail in cfgs:
                if tail is None:
                    os.environ.pop("GOL_TAIL", None)
                else:
                    os.environ["GOL_TAIL"] = tail
                e.set_tuning(band_rows=band, gens_per_pass=G)
                e.step(G, hashes=hashed)
                e.profile(True)
                e.profile_reset()
                t0 = time.perf_counter()
                e.step(n, hashes=hashed)
                e.sync()
                dt = time.perf_counter() - t0
                ms, _, _ = e.profile_read()
                clk = e.profile_clock()
                e.profile(False)
                k = W * H * n / (ms * 1e-3) / 1e9
                res[(band, tail)].append((k / clk, k, clk))
                print(f"{W}x{H} G={G}{' hashed' if hashed else ''} round{rnd} band={band or 'auto':>4} tail={tail or '-':>6} kernel_GCUPS={k:9.1f} "
                      f"clock={clk:.3f} per_GHz={k / clk:8.1f} wall_GCUPS={W * H * n / dt / 1e9:9.1f}", flush=True)
        os.environ.pop("GOL_TAIL", None)
    print("# summary: median per-GHz, median kernel GCUPS")
    for c, v in sorted(res.items(), key=lambda kv: -sorted(x[0] for x in kv[1])[1]):
        pg = sorted(x[0] for x in v)[1]
        kg = sorted(x[1] for x in v)[1]
        print(f"band={c[0] or 'auto':>4} tail={c[1] or '-':>6} per_GHz={pg:8.1f} kernel_GCUPS={kg:9.1f}")


if __name__ == "__main__":
    main()
