#!/usr/bin/env python3
"""Depth x band sweep on small tori (the pass planner's narrow-board rules
were measured at 65536^2; a 4096^2 pass of G = 10 in 256-row bands is only
32 waves).  Prints kernel and wall microseconds per generation for every
(edge, G, band); unhashed and hashed.

    python scripts/small_sweep.py [GENS]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife.engine import GolEngine  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 120
    edges = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1024, 2048, 4096, 8192, 16384, 32768]
    for S in edges:
        with GolEngine(S, S) as e:
            e.seed(0x5EED)
            e.step(50)
            e.sync()
            for hashed in (False, True):
                best = None
                for G in (1, 2, 3, 4, 5, 6, 8, 10):
                    for B in (2, 4, 6, 8, 12, 16, 24, 32, 64, 128, 256):
                        if G == 1 and B not in (4, 6, 8):
                            continue
                        e.set_tuning(band_rows=B, gens_per_pass=G)
                        e.step(2 * G, hashes=hashed)
                        e.sync()
                        e.profile(True)
                        e.profile_reset()
                        t0 = time.perf_counter()
                        e.step(n, hashes=hashed)
                        e.sync()
                        dt = time.perf_counter() - t0
                        ms, launches, gens = e.profile_read()
                        e.profile(False)
                        wall_us = dt * 1e6 / n
                        kern_us = ms * 1e3 / n
                        print(f"S={S:6d} hash={int(hashed)} G={G:2d} band={B:4d} wall_us/gen={wall_us:9.3f} "
                              f"kernel_us/gen={kern_us:9.3f} launches={launches} wall_GCUPS={S * S / wall_us / 1e3:9.1f}",
                              flush=True)
                        if best is None or wall_us < best[0]:
                            best = (wall_us, G, B)
                e.set_tuning()
                e.step(2 * 10, hashes=hashed)
                e.sync()
                t0 = time.perf_counter()
                e.step(n, hashes=hashed)
                e.sync()
                dt = time.perf_counter() - t0
                print(f"S={S:6d} hash={int(hashed)} BEST G={best[1]} band={best[2]} wall_us/gen={best[0]:.3f} "
                      f"({S * S / best[0] / 1e3:.1f} GCUPS); library auto plan {e.pass_plan(n, hashes=hashed)[:4]}... "
                      f"wall_us/gen={dt * 1e6 / n:.3f}", flush=True)


if __name__ == "__main__":
    main()
