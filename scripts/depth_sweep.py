#!/usr/bin/env python3
"""Time of one pass at each temporal-blocking depth G = 1..12 (reseeded board,
6 warm-up generations, 24 timed generations, min of ROUNDS interleaved rounds):
the cost table behind gol_step's pass planner.

    python scripts/depth_sweep.py [WxH ...]     env: ROUNDS=3  HASH=1 (fused hashes)  MAXG=12
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife.engine import GolEngine  # noqa: E402


def main():
    shapes = [tuple(int(x) for x in (a.split("x") if "x" in a else (a, a))) for a in sys.argv[1:]] or \
        [(262144, 262144), (262144, 32768), (65536, 65536)]
    rounds = int(os.environ.get("ROUNDS", "3"))
    hashes = os.environ.get("HASH", "0") == "1"
    maxg = int(os.environ.get("MAXG", "12"))
    for W, H in shapes:
        with GolEngine(W, H) as e:
            res = {}
            for _ in range(rounds):
                for G in range(1, maxg + 1):
                    gens = 24 if 24 % G == 0 else G * (24 // G + 1)
                    gens = max(gens, 2 * G)
                    e.set_tuning(gens_per_pass=G, words_per_lane=int(os.environ.get("WPL", "0")))
                    e.seed(0x5EED)
                    e.step(6)
                    e.profile(True)
                    e.profile_reset()
                    e.step(gens, hashes=hashes)
                    e.sync()
                    ms, n, g = e.profile_read()
                    e.profile(False)
                    res.setdefault(G, []).append(ms / n)
            base = min(res[6])
            for G in range(1, maxg + 1):
                t = min(res[G])
                print(f"shape={W}x{H} hash={int(hashes)} G={G} ms/pass={t:.4f} ms/gen={t / G:.4f} pass/pass(G=6)={t / base:.3f} "
                      f"GCUPS={W * H * G / t / 1e6:9.1f}", flush=True)


if __name__ == "__main__":
    main()
