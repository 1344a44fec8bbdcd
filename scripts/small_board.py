#!/usr/bin/env python3
"""Where the time of small boards goes: wall vs kernel time of gol_step on
boards from 1024^2 to 16384^2 (BASELINE.json configs[1] is 4096^2 x 1000
generations), unhashed and hashed, with the pass plan and the launches.

    python scripts/small_board.py [GENS]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife.engine import GolEngine  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    for S in (1024, 4096, 16384, 65536):
        with GolEngine(S, S) as e:
            e.seed(0x5EED)
            e.step(100)
            e.sync()
            for hashed in (False, True):
                for rep in range(2):
                    e.profile(True)
                    e.profile_reset()
                    t0 = time.perf_counter()
                    e.step(n, hashes=hashed)
                    e.sync()
                    dt = time.perf_counter() - t0
                    ms, launches, gens = e.profile_read()
                    e.profile(False)
                    print(f"{S:6d}^2 hash={int(hashed)} rep{rep} wall={dt * 1e3:9.3f} ms kernels={ms:9.3f} ms "
                          f"launches={launches} (us/launch wall {dt * 1e6 / max(launches, 1):7.2f}, kernel "
                          f"{ms * 1e3 / max(launches, 1):7.2f}) wall GCUPS={S * S * n / dt / 1e9:9.1f} "
                          f"kernel GCUPS={S * S * n / ms / 1e6:9.1f}", flush=True)
            # one generation per call: what a JVM worker calling step(1) per tick pays
            t0 = time.perf_counter()
            for _ in range(200):
                e.step(1)
            e.sync()
            dt = time.perf_counter() - t0
            print(f"{S:6d}^2 step(1) x 200: {dt * 1e6 / 200:8.2f} us per call, {S * S * 200 / dt / 1e9:9.1f} GCUPS",
                  flush=True)


if __name__ == "__main__":
    main()
