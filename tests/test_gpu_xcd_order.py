"""GPU: the step kernels' XCD-aware block order (gol_stencil.h xcd_block,
DESIGN.md §4 "Memory operations") only permutes which block runs which
(strip, band) tile: boards and per-generation hashes are bit-exact against
the oracle for any chunk, including chunks that leave a partial last group
and launches smaller than one group.  GOL_XCD_CHUNK is read once per
process, so each chunk runs in its own child process."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import json, sys
sys.path[:0] = [sys.argv[1], sys.argv[1] + '/akka-game-of-life_amd']
from gameoflife.engine import GolEngine
from oracle import oracle as O
W, H, gens, gpp = (int(x) for x in sys.argv[2:6])
board = O.seed_packed(W, H, 77)
with GolEngine(W, H, topology='torus', rule='life') as e:
    e.set_tuning(gens_per_pass=gpp)
    e.load(board)
    hs = e.step(gens, hashes=True)
    snap = e.snapshot()
print(json.dumps({'hashes': [int(h) for h in hs], 'crc': int(O.hash_packed(snap, W))}))
"""


@pytest.mark.parametrize("chunk", [1, 3, 8, 64])
@pytest.mark.parametrize("W,H,gpp", [(16384, 4096, 6), (65536, 2048, 1), (262144, 512, 7), (4096, 97, 3)])
def test_block_order_bit_exact(gpu, chunk, W, H, gpp):
    gens = 9
    env = dict(os.environ, GOL_XCD_CHUNK=str(chunk))
    out = subprocess.run([sys.executable, "-c", CHILD, ROOT, str(W), str(H), str(gens), str(gpp)],
                         env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    got = json.loads(out.stdout.strip().splitlines()[-1])
    final, want = O.run_packed(O.seed_packed(W, H, 77), W, gens, O.TORUS, O.LIFE)
    assert got["hashes"] == [int(h) for h in np.asarray(want)], f"chunk {chunk}"
    assert got["crc"] == O.hash_packed(final, W)
