"""GPU parity at the headline size: the 262144^2 torus of BASELINE.json
configs[3] (8 GiB per plane), stepped one automatic 6-generation pass as one
context (N = 1) and as an in-process group of 8 row shards of 32768 rows (the
N = 8 decomposition and its halo schedule), bit-exact against the
multithreaded CPU oracle: per-generation hashes and the final board."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

W = H = 262144
GENS = 6  # one pass at the automatic depth: the benchmark's kernel


@pytest.fixture(scope="module")
def oracle_run():
    board = O.seed_packed(W, H, 0x5EED)
    final, hashes = O.run_packed(board, W, GENS, O.TORUS, O.LIFE)
    del board
    return final, hashes


def test_full_size_262144_one_context(gpu, oracle_run):
    from gameoflife.engine import GolEngine
    final, want = oracle_run
    with GolEngine(W, H) as e:
        e.seed(0x5EED)
        got = e.step(GENS, hashes=True)
        np.testing.assert_array_equal(got, want)
        assert np.array_equal(e.snapshot(), final)
        e.seed(0x5EED)
        e.step(GENS)  # the benchmark's own path: no fused hash
        assert e.hash() == int(want[-1])


def test_full_size_262144_eight_shards(gpu, oracle_run):
    from gameoflife import _native as N
    from gameoflife.engine import GolEngine, ShardGroup
    final, want = oracle_run
    shards = []
    for r in range(8):
        row0, rows = N.shard_rows(H, r, 8)
        s = GolEngine(W, H, row0=row0, rows=rows)
        s.seed(0x5EED)
        shards.append(s)
    g = ShardGroup(shards)
    try:
        got = g.step(GENS, hashes=True)
        np.testing.assert_array_equal(got, want)
        for s in shards:
            assert np.array_equal(s.snapshot(), final[s.row0:s.row0 + s.rows]), s.row0
    finally:
        g.close()
        for s in shards:
            s.close()
