#!/usr/bin/env python3
"""Does a board allocated after a freed 262144^2 board step slower?  Times the
65536^2 pass (reseeded, 6 warm-up generations, 36 timed) fresh, after a
262144^2 engine was created + seeded + freed, and after one was only
created + freed."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife.engine import GolEngine  # noqa: E402


def timed(S=65536, gens=36, rounds=3):
    best = 1e30
    with GolEngine(S, S) as e:
        for _ in range(rounds):
            e.seed(0x5EED)
            e.step(6)
            e.profile(True)
            e.profile_reset()
            e.step(gens)
            e.sync()
            ms, _, g = e.profile_read()
            e.profile(False)
            best = min(best, ms / g)
    return S * S / best / 1e6


def big(seed):
    with GolEngine(262144, 262144) as b:
        if seed:
            b.seed(0x5EED)
            b.step(6)
            b.sync()


print(f"fresh                      {timed():9.1f} GCUPS", flush=True)
big(True)
print(f"after 262144^2 seeded+run  {timed():9.1f} GCUPS", flush=True)
print(f"again                      {timed():9.1f} GCUPS", flush=True)
big(False)
print(f"after 262144^2 alloc only  {timed():9.1f} GCUPS", flush=True)
