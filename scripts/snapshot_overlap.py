#!/usr/bin/env python3
"""Periodic snapshots while stepping: every K generations the board goes to
the host, synchronously (gol_snapshot) or in the background
(gol_snapshot_async, page-locked buffer, waited for before the next one),
beside plain stepping.  Wall-clock GCUPS over R periods, best of ROUNDS.

    python scripts/snapshot_overlap.py [WxH ...]   env: K=120 R=6 ROUNDS=2
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife.engine import GolEngine  # noqa: E402


MODES = os.environ.get("MODES", "plain,sync,async").split(",")


def main():
    shapes = [tuple(int(x) for x in a.split("x")) for a in sys.argv[1:]] or [(65536, 65536), (262144, 262144)]
    K, R, rounds = (int(os.environ.get(k, d)) for k, d in (("K", "120"), ("R", "6"), ("ROUNDS", "2")))
    for W, H in shapes:
        with GolEngine(W, H) as e:
            pinned = e.host_buffer()
            pinned2 = e.host_buffer()
            best = {}
            for _ in range(rounds):
                for mode in MODES:
                    if mode.startswith("async"):
                        os.environ["GOL_SNAP_CHUNK_MB"] = mode.split("_")[1] if "_" in mode else "256"
                    e.seed(0x5EED)
                    e.step(K)
                    e.sync()
                    t0 = time.perf_counter()
                    t_call = 0.0
                    bufs = [pinned, pinned2]
                    for i in range(R):
                        e.step(K)
                        if mode == "sync":
                            e.snapshot(out=pinned)
                        elif mode.startswith("async"):
                            if i:
                                e.snapshot_wait()
                            tc = time.perf_counter()
                            e.snapshot_async(bufs[i % 2])
                            t_call += time.perf_counter() - tc
                    if mode.startswith("async"):
                        e.snapshot_wait()
                    e.sync()
                    dt = time.perf_counter() - t0
                    best[mode] = min(best.get(mode, 1e30), dt)
                    if mode.startswith("async"):
                        best["async_call_ms"] = t_call / R * 1e3
            plane = W * H / 8 / 2**30
            print(f"{W}x{H} snapshot_async call (host time) {best.pop('async_call_ms'):.3f} ms", flush=True)
            for mode, dt in best.items():
                print(f"{W}x{H} K={K} R={R} {mode:5s} {dt * 1e3:9.2f} ms  {W * H * K * R / dt / 1e9:9.1f} GCUPS "
                      f"(one {plane:.2f} GiB snapshot per {K} generations)", flush=True)


if __name__ == "__main__":
    main()
