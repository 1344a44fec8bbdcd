#!/usr/bin/env python3
"""Kernel time of consecutive 8-generation launches right after a context is
created, and again after the GPU idles: does the rate follow the clock's
ramp rather than the board?  (262144 x 32768 and 262144^2 by default.)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife.engine import GolEngine  # noqa: E402


def curve(e, n, label):
    out = []
    for _ in range(n):
        e.profile(True)
        e.profile_reset()
        e.step(8)
        e.sync()
        ms, _, _ = e.profile_read()
        e.profile(False)
        out.append(ms)
    print(f"{label:40s} " + " ".join(f"{x:.3f}" for x in out), flush=True)


def main():
    for W, H in [(262144, 32768), (262144, 262144)]:
        with GolEngine(W, H) as e:
            e.set_tuning(gens_per_pass=8)
            e.seed(0x5EED)
            curve(e, 24, f"{W}x{H} fresh context")
            e.seed(0x5EED)
            curve(e, 24, f"{W}x{H} reseeded, GPU busy")
            time.sleep(1.0)
            e.seed(0x5EED)
            curve(e, 24, f"{W}x{H} reseeded after 1 s idle")
            time.sleep(1.0)
            curve(e, 24, f"{W}x{H} evolved board after 1 s idle")


if __name__ == "__main__":
    main()
