#!/usr/bin/env python3
"""Pass depth on small tori under the small-board band rule (band_rows
automatic, gol_schedule.cpp small_board_band): for every fixed depth G, the
wall and kernel microseconds per generation of N generations (default 1000,
configs[1]), unhashed and hashed, min of 3 runs; then the library's own plan.

    python scripts/small_depth.py [N] [EDGES]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife.engine import GolEngine  # noqa: E402


def timed(e, n, hashed, reps=3):
    best = None
    for _ in range(reps):
        e.profile(True)
        e.profile_reset()
        e.sync()
        t0 = time.perf_counter()
        e.step(n, hashes=hashed)
        e.sync()
        dt = time.perf_counter() - t0
        ms, launches, _ = e.profile_read()
        e.profile(False)
        if best is None or dt < best[0]:
            best = (dt, ms, launches)
    return best


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    edges = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1024, 2048, 4096, 8192, 16384, 32768]
    for S in edges:
        with GolEngine(S, S) as e:
            e.seed(0x5EED)
            e.step(50)
            e.sync()
            for hashed in (False, True):
                rows = []
                for G in (4, 5, 6, 7, 8, 9, 10, 11, 12):
                    e.set_tuning(gens_per_pass=G)
                    e.step(2 * G, hashes=hashed)
                    dt, ms, launches = timed(e, n, hashed)
                    rows.append((dt, G))
                    print(f"S={S:6d} hash={int(hashed)} G={G:2d} wall_us/gen={dt * 1e6 / n:8.3f} "
                          f"kernel_us/gen={ms * 1e3 / n:8.3f} launches={launches:4d} "
                          f"wall_GCUPS={S * S * n / dt / 1e9:9.1f}", flush=True)
                e.set_tuning()
                e.step(20, hashes=hashed)
                dt, ms, launches = timed(e, n, hashed)
                best = min(rows)
                plan = e.pass_plan(n, hashes=hashed)
                print(f"S={S:6d} hash={int(hashed)} AUTO plan={plan[:3]}..x{len(plan)} wall_us/gen={dt * 1e6 / n:8.3f} "
                      f"kernel_us/gen={ms * 1e3 / n:8.3f} | best fixed G={best[1]} wall_us/gen={best[0] * 1e6 / n:8.3f}",
                      flush=True)


if __name__ == "__main__":
    main()
