#!/usr/bin/env python3
"""65536^2 (17 column strips: a pass is ~1-2 rounds of resident tiles) at
fixed (depth, band) pairs on a board that keeps evolving, interleaved rounds:
for each round and config, 48 untimed generations then 240 timed ones (a
multiple of 6, 8, 10 and 12); kernel time from the library's HIP events and
wall time.  Band 0 = the library's choice (with its tail split).

    python scripts/narrow_band_depth.py [--shape WxH] [--rounds R] 8:0 12:384 ...
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife.engine import GolEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="65536x65536")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("configs", nargs="+")
    a = ap.parse_args()
    W, H = (int(x) for x in a.shape.split("x"))
    cfgs = [tuple(int(v) for v in c.split(":")) for c in a.configs]
    res = {c: [] for c in cfgs}
    timed = 240
    with GolEngine(W, H) as e:
        e.seed(0x5EED)
        e.step(96)
        for r in range(a.rounds):
            for G, band in cfgs:
                e.set_tuning(band_rows=band, gens_per_pass=G)
                e.step(48)
                e.sync()
                e.profile(True)
                e.profile_reset()
                t0 = time.perf_counter()
                e.step(timed)
                e.sync()
                dt = time.perf_counter() - t0
                ms, n, g = e.profile_read()
                e.profile(False)
                res[(G, band)].append((W * H * timed / dt / 1e9, W * H * g / (ms / 1e3) / 1e9))
                print(f"{a.shape} r{r + 1} G={G:2d} band={band:4d} wall {res[(G, band)][-1][0]:9.1f} GCUPS  "
                      f"kernel {res[(G, band)][-1][1]:9.1f} GCUPS", flush=True)
    print("# summary: median wall GCUPS, median kernel GCUPS")
    for (G, band), v in res.items():
        print(f"G={G:2d} band={band:4d} {statistics.median(x[0] for x in v):9.1f} {statistics.median(x[1] for x in v):9.1f}")


if __name__ == "__main__":
    main()
