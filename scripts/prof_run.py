#!/usr/bin/env python3
"""Minimal workload driver for rocprofv3 counter passes: seed a torus board,
warm up, then run `gens` generations of B3/S23 at the given pass depth.

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch --output-format csv -- \
        python3 scripts/prof_run.py 262144 60 6
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife.engine import GolEngine  # noqa: E402


def main():
    edge = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    gens = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    gpp = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    with GolEngine(edge, edge) as e:
        e.set_tuning(gens_per_pass=gpp)
        e.seed(0x5EED)
        e.step(gens)
        e.sync()
    print(f"prof_run: {edge}^2 torus, {gens} generations, gens_per_pass={gpp or 'auto'}", flush=True)


if __name__ == "__main__":
    main()
