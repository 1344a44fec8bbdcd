#!/usr/bin/env python3
"""Single-generation passes (default 65536^2) by band height (and lane width), the
way bench.py times its single_generation_passes line: seed, 50 ms of untimed
steps, then 256 timed generations; kernel time (HIP events) and wall time.
Interleaved rounds in one process.

    python scripts/g1_band_path.py [--rounds R] 4:4 6:4 8:4 ...   (band:words_per_lane)
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shape", default="65536x65536")
    ap.add_argument("--gens", type=int, default=256)
    ap.add_argument("configs", nargs="+")
    a = ap.parse_args()
    cfgs = [tuple(int(v) for v in c.split(":")) for c in a.configs]
    res = {c: [] for c in cfgs}
    W, H = (int(x) for x in a.shape.split("x"))
    algo = W * H * 0.25
    with GolEngine(W, H) as e:
        for r in range(a.rounds):
            for band, vec in cfgs:
                e.set_tuning(band_rows=band, gens_per_pass=1, words_per_lane=vec)
                e.seed(0x5EED)
                t0 = time.perf_counter()
                while (time.perf_counter() - t0) < 0.05:
                    e.step(16)
                    e.sync()
                e.profile(True)
                e.profile_reset()
                t0 = time.perf_counter()
                e.step(a.gens)
                e.sync()
                dt = time.perf_counter() - t0
                ms, n, g = e.profile_read()
                e.profile(False)
                kms = ms / n
                res[(band, vec)].append((algo / (kms / 1e3) / 8e12, algo / (dt / a.gens) / 8e12, kms))
                print(f"r{r + 1} band={band} vec={vec} kernel {kms:.4f} ms  frac {res[(band, vec)][-1][0]:.4f}  "
                      f"wall frac {res[(band, vec)][-1][1]:.4f}", flush=True)
    print("# summary: median HBM fraction by kernel time / by wall time, median kernel ms")
    for (band, vec), v in res.items():
        print(f"band={band} vec={vec} {statistics.median(x[0] for x in v):.4f} {statistics.median(x[1] for x in v):.4f} "
              f"{statistics.median(x[2] for x in v):.4f}")


if __name__ == "__main__":
    main()
