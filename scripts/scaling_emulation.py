#!/usr/bin/env python3
"""What each rank of an N-GPU run of the bench computes, on one GPU: the
262144^2 board whole (N = 1) and one rank's row block of it for N = 2, 4, 8
(262144 x 262144/N, stepped as a 1-rank RCCL self-ring: the sharded pass's
interior launch, G-row halo send/recv, boundary rows).  Interleaved rounds;
per shape the driver's window (seed, 5 warm-up generations, 20 timed, wall
clock) and the same after 50 ms of untimed steps.  rate(N) / rate(1) is the
per-cell efficiency an N-GPU run can reach before any xGMI cost (the bench's
value at N = (W*H*K) / max-over-ranks time).

    python scripts/scaling_emulation.py [--rounds R]
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife import _native as N  # noqa: E402
from gameoflife.engine import GolEngine  # noqa: E402

W = 262144


def window(e, settle_ms):
    e.seed(0x5EED)
    if settle_ms:
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < settle_ms:
            e.step(12)
            e.sync()
        e.seed(0x5EED)
    e.step(5)
    e.sync()
    t0 = time.perf_counter()
    e.step(20)
    e.sync()
    return W * e.rows * 20 / (time.perf_counter() - t0) / 1e9


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    engs = {}
    for n in (1, 2, 4, 8):
        if n == 1:
            engs[n] = GolEngine(W, W)
        else:
            engs[n] = GolEngine(W, W, row0=0, rows=W // n)
            engs[n].comm_init(N.unique_id(), 0, 1)
    res = {(n, s): [] for n in engs for s in (0, 50)}
    for r in range(a.rounds):
        for s in (0, 50):
            for n, e in engs.items():
                g = window(e, s)
                res[(n, s)].append(g)
                print(f"r{r + 1} N={n} settle={s:2d}ms rows={e.rows:6d} {g:9.1f} GCUPS", flush=True)
    print("# summary: median GCUPS per shape, and / N = 1 (per-cell efficiency before xGMI cost)")
    for s in (0, 50):
        base = statistics.median(res[(1, s)])
        for n in engs:
            m = statistics.median(res[(n, s)])
            print(f"settle={s:2d}ms N={n} rows={W // n:6d} {m:9.1f} GCUPS  eff={m / base:.3f}")
    for e in engs.values():
        e.close()


if __name__ == "__main__":
    main()
