#!/usr/bin/env python3
"""Host<->device cost of the boundary's board transfers (gol_load,
gol_snapshot: hipMemcpy2DAsync between the caller's row-major buffer and
the padded device plane, plus the pair-layout conversion kernel), from
pageable numpy buffers and from pinned host memory, and the PCIe-inclusive
rate of a step workload that uploads the board, runs N generations and
snapshots it (bench.py's `value` excludes these copies).

    python scripts/pcie_rate.py [edge ...]        (default 65536 262144)
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "akka-game-of-life_amd")]

import torch  # noqa: E402  (pinned host memory only)
from gameoflife.engine import GolEngine  # noqa: E402


def timed(fn, reps=3):
    best = 1e30
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        best = min(best, time.perf_counter() - t0)
    return best


def main():
    edges = [int(a) for a in sys.argv[1:]] or [65536, 262144]
    for S in edges:
        with GolEngine(S, S, topology="torus", rule="life") as e:
            nbytes = S * S // 8
            pageable = np.zeros((S, S // 32), dtype=np.uint32)
            pageable[::7, ::3] = 0x9E3779B9
            pinned_t = torch.empty((S, S // 32), dtype=torch.int32, pin_memory=True)
            pinned = pinned_t.numpy().view(np.uint32)
            pinned[:] = pageable
            t_fresh = timed(lambda: e.snapshot())
            print(f"{S}^2 snapshot into a fresh numpy array {t_fresh * 1e3:8.1f} ms "
                  f"({nbytes / t_fresh / 1e9:5.1f} GB/s: first-touch page faults)", flush=True)
            for name, buf in (("pageable", pageable), ("pinned", pinned)):
                e.load(buf)
                e.sync()
                t_load = timed(lambda: (e.load(buf), e.sync()))
                t_snap = timed(lambda: e.snapshot(out=buf))
                print(f"{S}^2 {name:8s} load {t_load * 1e3:8.1f} ms ({nbytes / t_load / 1e9:5.1f} GB/s)  "
                      f"snapshot into it {t_snap * 1e3:8.1f} ms ({nbytes / t_snap / 1e9:5.1f} GB/s)", flush=True)
            e.seed(0x5EED)
            e.step(12)
            e.sync()
            gens = 60
            t0 = time.perf_counter()
            e.step(gens)
            e.sync()
            t_step = time.perf_counter() - t0
            t_load = timed(lambda: (e.load(pinned), e.sync()), 1)
            t_snap = timed(lambda: e.snapshot(out=pinned), 1)
            gcups = S * S * gens / t_step / 1e9
            incl = S * S * gens / (t_step + t_load + t_snap) / 1e9
            print(f"{S}^2 {gens} generations: {gcups:.0f} GCUPS HBM-resident, {incl:.0f} GCUPS with a pinned "
                  f"upload + snapshot around them; one upload + snapshot = "
                  f"{(t_load + t_snap) / (t_step / gens):.0f} generations of compute", flush=True)
            del pinned, pinned_t


if __name__ == "__main__":
    main()
