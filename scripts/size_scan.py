#!/usr/bin/env python3
"""Per-cell rate of the planned B3/S23 passes across board shapes at a fixed
amount of work per run, with the in-kernel clock probe: separates a width
(row pitch, strips) effect from a size (plane bytes, power) effect.

    python scripts/size_scan.py [GENS_AT_262144^2]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife.engine import GolEngine  # noqa: E402

SHAPES = [(65536, 65536), (131072, 131072), (262144, 65536), (65536, 262144), (131072, 262144),
          (262144, 131072), (262144, 262144), (196608, 196608)]


def main():
    g_full = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    for W, H in SHAPES:
        n = max(10, int(round(g_full * (262144 * 262144) / (W * H) / 10)) * 10)
        with GolEngine(W, H) as e:
            e.seed(0x5EED)
            e.step(20)
            e.sync()
            for rep in range(3):
                e.profile(True)
                e.profile_reset()
                t0 = time.perf_counter()
                e.step(n)
                e.sync()
                dt = time.perf_counter() - t0
                ms, launches, _ = e.profile_read()
                clk = e.profile_clock()
                e.profile(False)
                print(f"{W}x{H} rep{rep} gens={n} wall_GCUPS={W * H * n / dt / 1e9:9.1f} "
                      f"kernel_GCUPS={W * H * n / (ms * 1e-3) / 1e9:9.1f} clock_GHz={clk:.3f} "
                      f"GCUPS_per_GHz={W * H * n / (ms * 1e-3) / 1e9 / max(clk, 1e-9):8.1f} "
                      f"plan={e.pass_plan(n)[:2]}", flush=True)


if __name__ == "__main__":
    main()
