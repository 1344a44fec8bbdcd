"""Child process of tests/test_gpu_quads.py (not a test module): libgol and
the oracle with GOL_LAYOUT=quads set before either is loaded, so every torus
whose rows hold whole quads of words runs the quad layout -- the seed,
load / snapshot conversions, gol_get_cell, the quad kernels (step_kernel<4>,
multistep_hg_kernel<4> up to 8 generations per pass, multistep_kernel<4>
deeper and for generic rules) and the quad hash -- checked bit-exact against
the oracle, which follows the same switch.  Prints one line per check and
"QUADS OK" at the end."""
import os
import sys
import threading
import uuid

os.environ["GOL_LAYOUT"] = "quads"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

import numpy as np  # noqa: E402

from gameoflife import _native as N  # noqa: E402
from gameoflife.engine import GolEngine  # noqa: E402
from gameoflife.rules import Rule  # noqa: E402
from oracle import oracle as O  # noqa: E402


def log(*a):
    print(*a, flush=True)


def run_check(W, H, gens, rule=O.LIFE, gpp=0, hashed=True, seed=1, band=0):
    board = O.seed_packed(W, H, seed)
    with GolEngine(W, H, topology="torus", rule=Rule(*rule)) as e:
        e.set_tuning(band_rows=band, gens_per_pass=gpp)
        e.load(board)
        assert e.hash() == O.hash_packed(board, W)
        got = e.step(gens, hashes=hashed)
        h = e.hash()
        final = e.snapshot()
    ref, want = O.run_packed(board, W, gens, O.TORUS, rule)
    np.testing.assert_array_equal(final, ref)
    assert h == int(want[-1])
    if hashed:
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, f"{W}x{H} G={gpp}: first hash mismatch at generation {bad[0] + 1}"


def main():
    assert N.device_layout(32 * 8) == 4 and N.device_layout(32 * 6) == 2 and O.device_ilv(32 * 8) == 4
    # layout, seed, conversions, get_cell
    W, H = 4096, 64
    with GolEngine(W, H) as e:
        e.seed(0x5EED)
        b = O.seed_packed(W, H, 0x5EED)
        np.testing.assert_array_equal(e.snapshot(), b)
        assert e.hash() == O.hash_packed(b, W)
        cells = O.unpack(b, W)
        for x, y in [(0, 0), (1, 0), (3, 5), (4, 5), (127, 9), (128, 9), (4095, 63), (2050, 31)]:
            assert e.get_cell(x, y) == bool(cells[y, x]), (x, y)
        assert e.occupancy(8)[1] == 248 and e.occupancy(12)[1] == 248 and e.occupancy(1)[1] == 256
    log("layout / seed / snapshot / get_cell ok")
    # hashed runs at every depth, partial strips
    for gpp in (1, 2, 3, 5, 7, 8, 9, 10, 12):
        run_check(32 * 260, 37, 9, gpp=gpp, seed=gpp)
        run_check(32 * 12, 29, 9, gpp=gpp, seed=gpp + 50)
    log("hashed depths ok")
    # unhashed, every depth, strip edges of the 248-word quad strip
    for words in (4, 60, 124, 244, 248, 252, 492, 496, 500, 1024):
        for gpp in range(1, 13):
            run_check(32 * words, 2 * gpp + 7, 2 * gpp + 1, gpp=gpp, hashed=False, seed=words * 13 + gpp)
    log("unhashed depths ok")
    # band heights, generic rules (vertical-first quads, depth capped at 7)
    for band in (1, 3, 16, 1000):
        run_check(32 * 248, 61, 14, gpp=7, band=band, seed=band)
    for rule in ((0x0C8, 0x1A6), (0x049, 0x16E), O.REF_LITERAL):
        for gpp in (0, 2, 7, 12):
            run_check(32 * 132, 31, 9, rule=rule, gpp=gpp, seed=gpp)
    log("bands / generic rules ok")
    # the BASELINE config-2 board, 1000 generations at the planner's passes
    b = O.seed_packed(4096, 4096, 7)
    with GolEngine(4096, 4096) as e:
        e.load(b)
        got = e.step(1000, hashes=True)
    _, want = O.run_packed(b, 4096, 1000)
    np.testing.assert_array_equal(got, want)
    log("4096^2 x 1000 ok")
    # the ring schedule: 2 loopback ranks, 8-generation passes
    W, H = 32 * 128, 40
    board = O.seed_packed(W, H, 4242)
    key = uuid.uuid4().hex
    engs = []
    for r in range(2):
        row0, rows = N.shard_rows(H, r, 2)
        e = GolEngine(W, H, row0=row0, rows=rows)
        e.set_tuning(gens_per_pass=8)
        e.load(board[row0:row0 + rows])
        e.comm_init_loopback(key, r, 2)
        engs.append(e)
    out = [None, None]

    def work(r):
        out[r] = engs[r].allreduce_u64(engs[r].step(16, hashes=True))

    ts = [threading.Thread(target=work, args=(r,)) for r in range(2)]
    [t.start() for t in ts]
    [t.join(120) for t in ts]
    final = np.vstack([e.snapshot() for e in engs])
    for e in engs:
        e.close()
    ref, want = O.run_packed(board, W, 16)
    np.testing.assert_array_equal(out[0], want)
    np.testing.assert_array_equal(final, ref)
    log("loopback ring ok")
    log("QUADS OK")


if __name__ == "__main__":
    main()
