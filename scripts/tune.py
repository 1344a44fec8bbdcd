#!/usr/bin/env python3
"""Sweep of lane width x pass depth G x band size for the step kernel:
interleaved rounds in one process, kernel time from HIP events.

    python scripts/tune.py [edge | WxH ...]
    env: VECS=4  GPPS=1,2,3,4  BANDS=0,16,...  ROUNDS=3  HASH=1
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife.engine import GolEngine  # noqa: E402


def measure(e, gens, hashes=False):
    e.profile(True)
    e.profile_reset()
    t0 = time.perf_counter()
    e.step(gens, hashes=hashes)
    e.sync()
    wall = time.perf_counter() - t0
    ms, n, g = e.profile_read()
    e.profile(False)
    return ms / max(g, 1), wall / gens * 1e3  # kernel ms per generation, wall ms per generation


def parse_shape(s):
    if "x" in s:
        w, h = s.split("x")
        return int(w), int(h)
    return int(s), int(s)


def main():
    shapes = [parse_shape(a) for a in sys.argv[1:]] or [(65536, 65536), (262144, 262144)]
    bands = [int(b) for b in os.environ.get("BANDS", "0,16,32,64,128,256").split(",")]
    gpps = [int(g) for g in os.environ.get("GPPS", "1,2,3,4").split(",")]
    rounds = int(os.environ.get("ROUNDS", "3"))
    vecs = [int(v) for v in os.environ.get("VECS", "4").split(",")]
    hashes = os.environ.get("HASH", "1") == "1"
    for (W, H) in shapes:
        gens = 48 if W * H <= 65536 * 65536 else 12
        with GolEngine(W, H) as e:
            e.seed(0x5EED)
            e.step(3)
            keys = [(v, g, b) for v in vecs for g in gpps for b in bands]
            res = {k: [] for k in keys}
            resh = {k: [] for k in keys}
            for _ in range(rounds):
                for key in keys:
                    v, g, b = key
                    e.set_tuning(band_rows=b, gens_per_pass=g, words_per_lane=v)
                    res[key].append(measure(e, gens))
                    if hashes:
                        resh[key].append(measure(e, gens, hashes=True))
            bytes_per_gen = W * H * 0.25
            for key in keys:
                v, g, b = key
                e.set_tuning(band_rows=b, gens_per_pass=g, words_per_lane=v)
                occ = e.occupancy(g)
                k = min(x[0] for x in res[key])
                med = sorted(x[0] for x in res[key])[len(res[key]) // 2]
                w = min(x[1] for x in res[key])
                kh = min(x[0] for x in resh[key]) if hashes else float("nan")
                print(f"shape={W}x{H} VEC={v} G={g} band={b:5d} kernel_ms/gen={k:.4f} median={med:.4f} "
                      f"wall_ms/gen={w:.4f} GCUPS={W * H / k / 1e6:9.1f} "
                      f"frac={bytes_per_gen / k / 1e6 / 8000:.3f} waves/CU={occ[0]} strip={occ[1]} | "
                      f"hash: kernel_ms/gen={kh:.4f} frac={bytes_per_gen / kh / 1e6 / 8000:.3f}", flush=True)


if __name__ == "__main__":
    main()
