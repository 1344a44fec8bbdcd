#!/usr/bin/env python3
"""Single-generation passes (the pure-bandwidth case) at 65536^2: kernel
time per generation over band heights x lane widths, beside the device-to-
device copy rate of the same bytes (torch copy_, 512 MiB read + 512 MiB
written per 'generation').

    python scripts/g1_sweep.py      env: BANDS=16,64,128  VECS=2,4  ROUNDS=3
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

import torch  # noqa: E402

from gameoflife.engine import GolEngine  # noqa: E402

S = 65536


def copy_rate(rounds):
    a = torch.empty(S * S // 8, dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    best = 1e30
    for _ in range(rounds):
        b.copy_(a)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            b.copy_(a)
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / 20)
    return best * 1e3, 2 * a.numel() / best / 1e9


def main():
    bands = [int(x) for x in os.environ.get("BANDS", "0,16,64,128").split(",")]
    vecs = [int(x) for x in os.environ.get("VECS", "2,4").split(",")]
    rounds = int(os.environ.get("ROUNDS", "3"))
    ms, gbs = copy_rate(rounds)
    print(f"copy_ 512 MiB -> 512 MiB: {ms:.4f} ms = {gbs:.0f} GB/s (one generation's algorithmic bytes)", flush=True)
    with GolEngine(S, S) as e:
        res = {}
        for _ in range(rounds):
            for v in vecs:
                for b in bands:
                    e.set_tuning(band_rows=b, gens_per_pass=1, words_per_lane=v)
                    e.seed(0x5EED)
                    e.step(4)
                    e.profile(True)
                    e.profile_reset()
                    e.step(40)
                    e.sync()
                    k, _, g = e.profile_read()
                    e.profile(False)
                    res.setdefault((v, b), []).append(k / g)
        for (v, b), xs in sorted(res.items()):
            k = min(xs)
            print(f"G=1 VEC={v} band={b:4d} kernel_ms/gen={k:.4f} GCUPS={S * S / k / 1e6:8.1f} "
                  f"algorithmic={S * S / 4 / k / 1e6:6.0f} GB/s frac={S * S / 4 / k / 1e6 / 8000:.3f}", flush=True)


if __name__ == "__main__":
    main()
