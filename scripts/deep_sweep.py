#!/usr/bin/env python3
"""Per-generation time at fixed temporal-blocking depths, on a board that keeps
evolving (no reseed between depths) with the GPU kept busy: for each round and
depth G, 48 untimed generations then 120 timed ones (a multiple of 6, 8, 10
and 12), kernel time from the library's HIP events.  Min over rounds.

    GOL_LIB_PATH=ab/deep/lib/libgol.so python scripts/deep_sweep.py [WxH ...]
    env: DEPTHS="6 8 10 12"  ROUNDS=3  HASH=1
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife.engine import GolEngine  # noqa: E402


def main():
    shapes = [tuple(int(x) for x in (a.split("x") if "x" in a else (a, a))) for a in sys.argv[1:]] or \
        [(262144, 262144), (65536, 65536)]
    depths = [int(g) for g in os.environ.get("DEPTHS", "6 8 10 12").split()]
    rounds = int(os.environ.get("ROUNDS", "3"))
    hashes = os.environ.get("HASH", "0") == "1"
    timed = 120
    for W, H in shapes:
        with GolEngine(W, H) as e:
            e.seed(0x5EED)
            e.step(96)
            res = {}
            for _ in range(rounds):
                for G in depths:
                    e.set_tuning(gens_per_pass=G)
                    e.step(48, hashes=hashes)
                    e.profile(True)
                    e.profile_reset()
                    e.step(timed, hashes=hashes)
                    e.sync()
                    ms, n, g = e.profile_read()
                    e.profile(False)
                    res.setdefault(G, []).append(ms / g)
            ref = min(res[8]) if 8 in res else min(min(v) for v in res.values())
            for G in depths:
                t = min(res[G])
                print(f"{W}x{H} hash={int(hashes)} G={G:2d} ms/gen={t:.5f} rel_G8={t / ref:.4f} "
                      f"GCUPS={W * H / t / 1e6:9.1f}  rounds={' '.join(f'{x:.5f}' for x in res[G])}", flush=True)


if __name__ == "__main__":
    main()
