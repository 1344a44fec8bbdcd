#!/usr/bin/env python3
"""Same-box A/B of explicit pass mixes (each pass run at a fixed
gens_per_pass) on the bench's fresh board: reseed, a 5-generation warm-up,
then the timed passes; interleaved rounds (DESIGN.md "Pass planner").

    python scripts/plan_mix_ab.py [--shape WxH] [--rounds R] [--hash] 6,6,8 10,10 8,12 ...
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife.engine import GolEngine  # noqa: E402


def run(e, plan, hashed):
    e.seed(0x5EED)
    e.set_tuning(gens_per_pass=0)
    e.step(5, hashes=hashed)
    e.sync()
    t0 = time.perf_counter()
    for g in plan:
        e.set_tuning(gens_per_pass=g)
        e.step(g, hashes=hashed)
    e.sync()
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="262144x262144")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--hash", action="store_true")
    ap.add_argument("plans", nargs="+")
    a = ap.parse_args()
    W, H = (int(x) for x in a.shape.split("x"))
    plans = {p: [int(g) for g in p.split(",")] for p in a.plans}
    with GolEngine(W, H) as e:
        for plan in plans.values():  # load every depth once
            run(e, plan, a.hash)
        best = {}
        for r in range(a.rounds):
            for name, plan in plans.items():
                dt = run(e, plan, a.hash)
                gc = W * H * sum(plan) / dt / 1e9
                best[name] = max(best.get(name, 0.0), gc)
                print(f"{a.shape} hash={int(a.hash)} r{r + 1} {name:12s} {dt * 1e3:8.3f} ms  {gc:9.1f} GCUPS", flush=True)
        for name, gc in best.items():
            print(f"{a.shape} hash={int(a.hash)} best {name:12s} {gc:9.1f} GCUPS", flush=True)


if __name__ == "__main__":
    main()
