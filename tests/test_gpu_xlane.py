"""GPU: the pair B3/S23 torus passes with their cross-lane words over the LDS
crossbar (multistep_bp_kernel, GOL_XLANE=lds -- VERDICT r04 item 2's
experiment) are bit-exact: every depth, partial and idle-lane strips, band
sizes, tiny heights and the 65536^2 board, final boards word for word and
gol_hash against the oracle.  The switch is read once per process, so the
checks run in a child process (one at a time, like the rest of the suite)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
import numpy as np
sys.path[:0] = [ROOT, ROOT + "/akka-game-of-life_amd"]
from oracle import oracle as O
from gameoflife.engine import GolEngine

def run(W, H, gens, gpp, band=0, seed=1):
    board = O.seed_packed(W, H, seed)
    with GolEngine(W, H, topology="torus", rule="life") as e:
        e.set_tuning(band_rows=band, gens_per_pass=gpp)
        e.load(board)
        e.step(gens)
        got, h = e.snapshot(), e.hash()
    final, want = O.run_packed(board, W, gens, O.TORUS, O.LIFE)
    assert np.array_equal(got, final), (W, H, gens, gpp, band)
    assert h == int(want[-1]), (W, H, gens, gpp, band)

for gpp in range(2, 13):
    run(32 * 300, 45, 2 * gpp + 1, gpp, seed=gpp)            # 3 strips, the last one partial (idle lanes)
for W in (32 * 2, 32 * 4, 32 * 124, 32 * 126, 32 * 248, 32 * 250):
    run(W, 33, 17, 7, seed=W)
for band in (1, 2, 5, 64, 1000):
    run(32 * 512, 130, 15, 7, band=band, seed=band)
for H in (1, 2, 3, 7):
    run(32 * 128, H, 9, 0, seed=H)
run(32 * 128, 97, 40, 0, seed=5)                            # the planner's depths
S = 65536
board = O.seed_packed(S, S, 0x5EED)
with GolEngine(S, S, topology="torus", rule="life") as e:
    e.set_tuning(gens_per_pass=7)
    e.seed(0x5EED)
    e.step(21)
    got = e.snapshot()
final, _ = O.run_packed(board, S, 21, O.TORUS, O.LIFE, want_hashes=False)
assert np.array_equal(got, final), "65536^2"
print("xlane ok")
""".replace("ROOT", repr(ROOT))


def test_lds_cross_lane_passes_bit_exact(gpu):
    env = dict(os.environ, GOL_XLANE="lds")
    p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0 and "xlane ok" in p.stdout, (p.stdout[-2000:], p.stderr[-3000:])
