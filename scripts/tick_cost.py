#!/usr/bin/env python3
"""Per-call cost of gol_step(1) with and without the per-generation hash
(the reference's per-tick drive, BoardCreator.scala:113-116) on the default
7 x 7 board and on 4096^2.

    python scripts/tick_cost.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife.engine import GolEngine  # noqa: E402


def main():
    for W, H, topo in ((7, 7, "ref-clipped"), (4096, 4096, "torus")):
        with GolEngine(W, H, topology=topo, rule="life") as e:
            e.seed(1)
            for hashed in (False, True):
                e.step(50, hashes=hashed)
                e.sync()
                t0 = time.perf_counter()
                for _ in range(500):
                    e.step(1, hashes=hashed)
                e.sync()
                dt = time.perf_counter() - t0
                print(f"{W}x{H} {topo} step(1) hash={int(hashed)}: {dt / 500 * 1e6:8.2f} us per call", flush=True)


if __name__ == "__main__":
    main()
