#!/usr/bin/env python3
"""Same-box A/B of band heights per pass depth on the bench's fresh board
(reseed, the 5-generation warm-up at the automatic plan, then the timed
passes, each at a fixed depth and band), interleaved rounds, in one process.
Run it with GOL_TAIL=1.0,3 so fixed bands keep the default tail split of wide
boards (gol_schedule.cpp tail_split).

    GOL_TAIL=1.0,3 python scripts/band_ab.py [--shape WxH] [--rounds R] 12:384,8:256 12:768,8:512 ...

A config "12:768,8:512" times a 12-generation pass in 768-row bands, then an
8-generation pass in 512-row bands (band 0 = the library's choice)."""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife.engine import GolEngine  # noqa: E402


def run(e, passes, hashed=False):
    e.seed(0x5EED)
    e.set_tuning()
    e.step(5, hashes=hashed)
    e.sync()
    e.profile(True)
    e.profile_reset()
    t0 = time.perf_counter()
    for g, band in passes:
        e.set_tuning(band_rows=band, gens_per_pass=g)
        e.step(g, hashes=hashed)
    e.sync()
    dt = time.perf_counter() - t0
    kms, _, _ = e.profile_read()
    clk = e.profile_clock()
    e.profile(False)
    return dt, kms / 1e3, clk


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="262144x262144")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--hash", action="store_true", help="fused per-generation hashes")
    ap.add_argument("--ring", action="store_true",
                    help="WxH is one rank's shard of a W x W board, stepped as a 1-rank RCCL self-ring")
    ap.add_argument("configs", nargs="+")
    a = ap.parse_args()
    W, H = (int(x) for x in a.shape.split("x"))
    cfgs = {c: [tuple(int(v) for v in p.split(":")) for p in c.split(",")] for c in a.configs}
    res = {c: [] for c in cfgs}
    eng = GolEngine(W, W, row0=0, rows=H) if a.ring else GolEngine(W, H)
    if a.ring:
        from gameoflife import _native as N
        eng.comm_init(N.unique_id(), 0, 1)
    with eng as e:
        for passes in cfgs.values():  # load every instance once
            run(e, passes, a.hash)
        for r in range(a.rounds):
            for name, passes in cfgs.items():
                dt, ks, clk = run(e, passes, a.hash)
                gens = sum(g for g, _ in passes)
                res[name].append((W * H * gens / dt / 1e9, W * H * gens / ks / 1e9, clk))
                print(f"{a.shape} h{int(a.hash)} r{r + 1} {name:20s} wall {dt * 1e3:8.3f} ms {res[name][-1][0]:9.1f} GCUPS  "
                      f"kernel {res[name][-1][1]:9.1f} GCUPS  clock {clk:.3f}", flush=True)
    print("# summary: median / max wall GCUPS, median kernel GCUPS, median clock")
    for name, v in res.items():
        print(f"{name:20s} {statistics.median(x[0] for x in v):9.1f} {max(x[0] for x in v):9.1f} "
              f"{statistics.median(x[1] for x in v):9.1f} {statistics.median(x[2] for x in v):.3f}")


if __name__ == "__main__":
    main()
