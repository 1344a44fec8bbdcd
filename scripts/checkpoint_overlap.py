#!/usr/bin/env python3
"""Fault-path checkpoints every K generations on an 8-shard in-process group
(one GPU): synchronous (gol_checkpoint) vs in the background
(gol_checkpoint_async into page-locked buffers), beside no checkpoints.

    python scripts/checkpoint_overlap.py [WxH]   env: K=48 GENS=480
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife.fault import ShardedSimulation  # noqa: E402


def main():
    W, H = (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "65536x65536").split("x"))
    K, gens = int(os.environ.get("K", "48")), int(os.environ.get("GENS", "480"))
    for rnd in range(2):
        for mode, every, asyn in (("none", 0, False), ("sync", K, False), ("async", K, True)):
            sim = ShardedSimulation(W, H, 8, [0], checkpoint_every=every, async_checkpoints=asyn)
            sim.step(K)  # warm-up (and the first buffers)
            t0 = time.perf_counter()
            sim.step(gens)
            sim._finish_checkpoint()  # the last background checkpoint lands inside the timed region
            for s in sim.shards:
                s.sync()
            dt = time.perf_counter() - t0
            sim.close()
            print(f"r{rnd} {W}x{H} 8 shards K={K} {mode:5s} {dt * 1e3:9.2f} ms  {W * H * gens / dt / 1e9:9.1f} GCUPS",
                  flush=True)


if __name__ == "__main__":
    main()
