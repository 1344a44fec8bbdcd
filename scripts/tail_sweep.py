#!/usr/bin/env python3
"""Band-schedule sweep (DESIGN.md section 4 "Band schedule"): kernel time per
generation for tail splits GOL_TAIL="frac,div" x bulk band heights,
interleaved rounds in one process (HIP-event time of the pass launches).
Every measurement reseeds the board and warms up 6 generations first: the
chip's clock follows the board's density (dense random boards draw more
power), so an evolving board would bias whatever is measured later.

    python scripts/tail_sweep.py [WxH ...]
    env: TAILS="0,0;1,2;..."  BANDS="0,256"  ROUNDS=3
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife.engine import GolEngine  # noqa: E402


def kernel_ms_per_gen(e, gens):
    e.profile(True)
    e.profile_reset()
    e.step(gens)
    e.sync()
    ms, _, g = e.profile_read()
    e.profile(False)
    return ms / max(g, 1)


def main():
    shapes = [tuple(int(x) for x in (a.split("x") if "x" in a else (a, a))) for a in sys.argv[1:]] or \
        [(65536, 65536), (262144, 32768), (262144, 262144)]
    tails = os.environ.get("TAILS", "0,0;0.5,2;1,2;1,3;2,2").split(";")
    bands = [int(b) for b in os.environ.get("BANDS", "0,256").split(",")]
    rounds = int(os.environ.get("ROUNDS", "3"))
    for W, H in shapes:
        gens = 36 if W * H <= 65536 * 65536 else 12
        with GolEngine(W, H) as e:
            keys = [(b, t) for b in bands for t in tails]
            res = {k: [] for k in keys}
            for _ in range(rounds):
                for b, t in keys:
                    os.environ["GOL_TAIL"] = t
                    e.set_tuning(band_rows=b)
                    e.seed(0x5EED)
                    e.step(6)
                    res[(b, t)].append(kernel_ms_per_gen(e, gens))
            os.environ.pop("GOL_TAIL", None)
            for b, t in keys:
                xs = sorted(res[(b, t)])
                print(f"shape={W}x{H} band={b:4d} tail={t:7s} kernel_ms/gen min={xs[0]:.4f} "
                      f"median={xs[len(xs) // 2]:.4f} GCUPS={W * H / xs[0] / 1e6:9.1f}", flush=True)


if __name__ == "__main__":
    main()
