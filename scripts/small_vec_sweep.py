#!/usr/bin/env python3
"""Small tori: 8-byte lanes (62-pair strips: a 4096^2 row of 64 pairs needs a
second strip that holds 2) against 16-byte lanes (the vertical-first kernel,
124 pairs per strip), depth x band.

    python scripts/small_vec_sweep.py [GENS]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife.engine import GolEngine  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 120
    for S in (2048, 4096, 8192, 16384, 32768):
        with GolEngine(S, S) as e:
            e.seed(0x5EED)
            e.step(50)
            e.sync()
            for wpl in (0, 4):
                for G in (4, 6, 8, 10):
                    for B in (2, 4, 8, 16, 32, 64):
                        e.set_tuning(band_rows=B, gens_per_pass=G, words_per_lane=wpl)
                        e.step(2 * G)
                        e.sync()
                        t0 = time.perf_counter()
                        e.step(n)
                        e.sync()
                        dt = time.perf_counter() - t0
                        print(f"S={S:6d} wpl={wpl} G={G:2d} band={B:3d} wall_us/gen={dt * 1e6 / n:9.3f} "
                              f"GCUPS={S * S * n / dt / 1e9:9.1f} occupancy={e.occupancy(G)}", flush=True)
            e.set_tuning()


if __name__ == "__main__":
    main()
