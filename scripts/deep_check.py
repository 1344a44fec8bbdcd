#!/usr/bin/env python3
"""Oracle check of a library build at fixed pass depths (default 9..12, the
experimental deep build ab/deep): per-generation hashes and final boards of
a few torus shapes.  Test infrastructure (imports oracle/).

    GOL_LIB_PATH=ab/deep/lib/libgol.so python scripts/deep_check.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))
sys.path.insert(0, ROOT)

from gameoflife.engine import GolEngine  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    depths = [int(g) for g in os.environ.get("DEPTHS", "9 10 11 12").split()]
    bad = 0
    for W, H, gens in [(32 * 520, 37, 25), (32 * 300, 45, 30), (4096, 200, 24), (32 * 2048, 40, 13)]:
        board = O.seed_packed(W, H, W + H)
        want_board, want = O.run_packed(board, W, gens, O.TORUS, O.LIFE)
        for G in depths:
            for hashed in (True, False):
                with GolEngine(W, H) as e:
                    e.set_tuning(gens_per_pass=G)
                    e.load(board)
                    got = e.step(gens, hashes=hashed)
                    snap = e.snapshot()
                    ok = np.array_equal(snap, want_board) and (not hashed or np.array_equal(got, want))
                    if hashed:
                        ok = ok and e.hash() == O.hash_packed(want_board, W)
                bad += not ok
                print(f"{W}x{H} gens={gens} G={G} hashed={hashed} {'ok' if ok else 'MISMATCH'}", flush=True)
    print("deep_check", "FAILED" if bad else "passed", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
