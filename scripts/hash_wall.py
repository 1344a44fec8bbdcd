#!/usr/bin/env python3
"""Wall time vs kernel time of hashed and unhashed gol_step calls at one
shape: where does a hashed step's time go outside the kernels?

    python scripts/hash_wall.py [W [H [GENS]]]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife.engine import GolEngine  # noqa: E402


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    H = int(sys.argv[2]) if len(sys.argv) > 2 else W
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    with GolEngine(W, H) as e:
        e.seed(0x5EED)
        e.step(6)
        e.sync()
        for label, hashed, gpp in [("unhashed auto", False, 0), ("hashed auto", True, 0), ("hashed G5", True, 5),
                                   ("hashed G6", True, 6), ("unhashed auto", False, 0), ("hashed auto", True, 0)]:
            e.set_tuning(gens_per_pass=gpp)
            e.step(n, hashes=hashed)
            e.sync()
            for rep in range(3):
                e.profile(True)
                e.profile_reset()
                t0 = time.perf_counter()
                e.step(n, hashes=hashed)
                e.sync()
                dt = time.perf_counter() - t0
                ms, launches, gens = e.profile_read()
                e.profile(False)
                print(f"{label:14s} rep{rep} plan={e.pass_plan(n, hashes=hashed)} wall={dt * 1e3:8.3f} ms "
                      f"kernels={ms:8.3f} ms ({launches} launches) wall GCUPS={W * H * n / dt / 1e9:9.1f} "
                      f"kernel GCUPS={W * H * n / ms / 1e6:9.1f}", flush=True)


if __name__ == "__main__":
    main()
