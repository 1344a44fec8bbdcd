#!/usr/bin/env python3
"""Minimal workload driver for rocprofv3 counter passes: seed a torus board,
run one warm-up pass, then `passes` passes of `G` generations (B3/S23).

    rocprofv3 --pmc FETCH_SIZE -T -d gpurun_out/pmc -o run --output-format csv -- \\
        python3 scripts/prof_run.py 262144x262144 8 [--passes 4] [--hash] [--ring]

G = 0 runs the pass planner on 60 generations instead (the bench's default).
--ring attaches a 1-rank RCCL communicator (the ring schedule: interior rows
launch + boundary rows launch per pass, halo rows sent to itself) -- the
per-rank launch shape of a row-sharded run.  Older form: `EDGE GENS GPP`.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife import _native as N  # noqa: E402
from gameoflife.engine import GolEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("shape")
    ap.add_argument("G", type=int)
    ap.add_argument("legacy_gpp", type=int, nargs="?", default=None)
    ap.add_argument("--passes", type=int, default=4)
    ap.add_argument("--hash", action="store_true")
    ap.add_argument("--ring", action="store_true")
    a = ap.parse_args()
    if "x" in a.shape:
        W, H = (int(v) for v in a.shape.split("x"))
        G, gens = a.G, (a.G * a.passes if a.G else 60)
    else:  # legacy: EDGE GENS GPP
        W = H = int(a.shape)
        gens, G = a.G, (a.legacy_gpp or 0)
    with GolEngine(W, H) as e:
        e.set_tuning(gens_per_pass=G)
        if a.ring:
            e.comm_init(N.unique_id(), 0, 1)
        e.seed(0x5EED)
        e.step(G or 6, hashes=a.hash)  # warm-up pass (the summariser skips it)
        e.step(gens, hashes=a.hash)
        e.sync()
    print(f"prof_run: {W}x{H} torus, {gens} generations, G={G or 'auto'} hash={int(a.hash)} "
          f"ring={int(a.ring)}", flush=True)


if __name__ == "__main__":
    main()
