#!/usr/bin/env python3
"""Cost of the sharded pass schedule on one GPU: a W x H torus stepped as one
context vs as an in-process group of k row shards (gol_group_*: interior
kernels || halo pulls, then boundary rows) on the same device.  The group's
kernels are exactly the RCCL-sharded ones, so the ratio bounds the per-pass
overhead a rank pays at N = k GPUs (minus the xGMI transfer itself).

    python scripts/shard_overhead.py [W] [H] [k] [gens]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife import _native as N  # noqa: E402
from gameoflife.engine import GolEngine, ShardGroup  # noqa: E402


def timed(step, sync, gens, rounds=3):
    step(6)
    sync()
    best = 1e30
    for _ in range(rounds):
        t0 = time.perf_counter()
        step(gens)
        sync()
        best = min(best, time.perf_counter() - t0)
    return best / gens * 1e3


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    gens = int(sys.argv[4]) if len(sys.argv) > 4 else 48
    with GolEngine(W, H) as e:
        e.seed(0x5EED)
        one = timed(lambda n: e.step(n), e.sync, gens)
    shards = []
    for r in range(k):
        row0, rows = N.shard_rows(H, r, k)
        s = GolEngine(W, H, row0=row0, rows=rows)
        s.seed(0x5EED)
        shards.append(s)
    g = ShardGroup(shards)
    grp = timed(lambda n: g.step(n), g.sync, gens)
    g.close()
    for s in shards:
        s.close()
    print(f"{W}x{H}: one context {one:.4f} ms/gen, group of {k} shards {grp:.4f} ms/gen, "
          f"overhead {100 * (grp / one - 1):.2f}%", flush=True)


if __name__ == "__main__":
    main()
