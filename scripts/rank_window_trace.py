#!/usr/bin/env python3
"""One N = 8 rank's driver window on this GPU, for a kernel trace: the
262144 x 32768 shard as a 1-rank RCCL self-ring (the ring schedule: interior
launch || halo send/recv, then boundary rows), seed, W = 5 warm-up and
K = 20 timed generations, twice.

    rocprofv3 --kernel-trace -d gpurun_out/rank -o rank --output-format csv -- \\
        python3 scripts/rank_window_trace.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife import _native as N  # noqa: E402
from gameoflife.engine import GolEngine  # noqa: E402


def main():
    W, rows = 262144, 32768
    with GolEngine(W, W, row0=0, rows=rows) as e:
        e.comm_init(N.unique_id(), 0, 1)
        for _ in range(2):
            e.seed(0x5EED)
            e.step(5)
            e.sync()
            t0 = time.perf_counter()
            e.step(20)
            e.sync()
            dt = time.perf_counter() - t0
            print(f"window: {dt * 1e3:.3f} ms, {W * rows * 20 / dt / 1e9:.1f} GCUPS", flush=True)


if __name__ == "__main__":
    main()
