#!/usr/bin/env python3
"""Same-box A/B of explicit pass mixes for 60 generations at 262144^2 (each
segment run at a fixed gens_per_pass): the planner's 4 x 7 + 4 x 8 against
2 x 6 + 6 x 8 and 7 x 8 + 4 (DESIGN.md "Pass planner").

    python scripts/plan_mix_ab.py [ROUNDS]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife.engine import GolEngine  # noqa: E402

MIXES = {"4x7+4x8": [(7, 28), (8, 32)], "2x6+6x8": [(6, 12), (8, 48)], "7x8+4": [(8, 56), (4, 4)],
         "10x6": [(6, 60)]}


def run(e, mix):
    e.seed(0x5EED)
    e.set_tuning(gens_per_pass=6)
    e.step(6)
    e.sync()
    t0 = time.perf_counter()
    for g, n in mix:
        e.set_tuning(gens_per_pass=g)
        e.step(n)
    e.sync()
    return time.perf_counter() - t0


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    W = H = 262144
    with GolEngine(W, H) as e:
        for mix in MIXES.values():  # load every depth once
            run(e, mix)
        for r in range(rounds):
            for name, mix in MIXES.items():
                dt = run(e, mix)
                print(f"r{r + 1} {name:8s} {dt * 1e3:8.3f} ms  {W * H * 60 / dt / 1e9:9.1f} GCUPS", flush=True)


if __name__ == "__main__":
    main()
