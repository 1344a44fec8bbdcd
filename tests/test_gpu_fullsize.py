"""GPU parity at the sizes and pass plans the benchmark times.

* 262144^2 torus (BASELINE.json configs[3], 8 GiB per plane), 20 generations
  -- the driver's `bench.py --steps 20`: the planner runs 10 + 10 unhashed
  and hashed (the wide G = 10 instances of multistep_hg_kernel with the
  row-pair-shared circuit, tail split active at >= 32 strips).
  As one context (N = 1), as an in-process group of 8 row shards of 32768 rows (the N = 8 decomposition:
  interior launch + boundary rows on the edge stream), and as a 1-rank RCCL
  self-ring (the ring schedule's ncclSend / ncclRecv).
* 65536^2 torus (configs[2]), 102 generations -- the kernels and pass depth
  of the bench's secondary run (7 x 10 + 2 x 9 + 2 x 7 unhashed; the bench
  times 101 x 10 + 2 x 7).
* 262144 x 16384: the benchmark's own unhashed path on a board of 67 strips
  with more than one round of resident waves (bulk bands + tail bands).

Everything is compared with the multithreaded CPU oracle: per-generation
hashes where the step fuses them, the final board word for word, and
gol_hash of the final board for the unhashed path."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

W = H = 262144
GENS = 20  # the driver's --steps 20


@pytest.fixture(scope="module")
def oracle_run():
    board = O.seed_packed(W, H, 0x5EED)
    final, hashes = O.run_packed(board, W, GENS, O.TORUS, O.LIFE)
    del board
    return final, hashes


def _unhashed_then_check(e, final, want_last):
    e.step(GENS)  # the benchmark's own path: no fused hash
    assert e.hash() == int(want_last)
    assert np.array_equal(e.snapshot(), final)


def test_full_size_262144_plans_are_the_benchs(gpu):
    from gameoflife.engine import GolEngine
    with GolEngine(W, H) as e:
        assert e.pass_plan(GENS) == [10, 10]
        assert e.pass_plan(GENS, hashes=True) == [10, 10]


def test_full_size_262144_one_context(gpu, oracle_run):
    from gameoflife.engine import GolEngine
    final, want = oracle_run
    with GolEngine(W, H) as e:
        e.seed(0x5EED)
        got = e.step(GENS, hashes=True)
        np.testing.assert_array_equal(got, want)
        assert np.array_equal(e.snapshot(), final)
        e.seed(0x5EED)
        _unhashed_then_check(e, final, want[-1])


def test_full_size_262144_self_ring(gpu, oracle_run):
    """The RCCL ring schedule on one GPU: a 1-rank communicator sends its
    first / last G rows to itself every pass (interior || exchange, then the
    boundary rows on the edge stream)."""
    from gameoflife import _native as N
    from gameoflife.engine import GolEngine
    final, want = oracle_run
    with GolEngine(W, H) as e:
        e.comm_init(N.unique_id(), 0, 1)
        e.seed(0x5EED)
        got = e.step(GENS, hashes=True)
        np.testing.assert_array_equal(e.allreduce_u64(got), want)
        e.seed(0x5EED)
        _unhashed_then_check(e, final, want[-1])


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
        for s in shards:
            s.seed(0x5EED)
        g.step(GENS)
        assert sum(s.hash() for s in shards) % (1 << 64) == int(want[-1])
        for s in shards:
            assert np.array_equal(s.snapshot(), final[s.row0:s.row0 + s.rows]), s.row0
    finally:
        g.close()
        for s in shards:
            s.close()


def test_full_size_65536_bench_plan(gpu):
    """configs[2]: the bench's secondary run's kernels, 102 generations
    (unhashed 7 x 10 + 2 x 9 + 2 x 7), final board and hash; hashed, every
    generation's hash."""
    from gameoflife.engine import GolEngine
    S, n = 65536, 102
    board = O.seed_packed(S, S, 0x5EED)
    final, want = O.run_packed(board, S, n, O.TORUS, O.LIFE)
    del board
    with GolEngine(S, S) as e:
        assert e.pass_plan(n) == [10] * 7 + [9, 9, 7, 7]
        e.seed(0x5EED)
        e.step(n)
        assert e.hash() == int(want[-1])
        assert np.array_equal(e.snapshot(), final)
        e.seed(0x5EED)
        got = e.step(n, hashes=True)
        np.testing.assert_array_equal(got, want)


def test_full_size_65536_single_generation_unhashed(gpu):
    """configs[2] one generation per pass without the hash -- exactly the
    bench's single_generation_passes instance (step_kernel<2, LIFE,
    HASH=false, pairs>, 4-row bands, non-temporal stores) -- final board word
    for word and gol_hash against the oracle."""
    from gameoflife.engine import GolEngine
    S, n = 65536, 8
    board = O.seed_packed(S, S, 0x5EED)
    final, want = O.run_packed(board, S, n, O.TORUS, O.LIFE)
    del board
    with GolEngine(S, S) as e:
        e.set_tuning(gens_per_pass=1)
        assert e.pass_plan(n) == [1] * n
        e.seed(0x5EED)
        e.step(n)
        assert e.hash() == int(want[-1])
        assert np.array_equal(e.snapshot(), final)


def test_wide_board_several_rounds_unhashed(gpu):
    """262144 x 16384 (67 strips, > 1 round of resident waves, tail bands):
    the unhashed planner path the headline times, against the oracle."""
    from gameoflife.engine import GolEngine
    Wd, Hd, n = 262144, 16384, 20
    board = O.seed_packed(Wd, Hd, 77)
    final, want = O.run_packed(board, Wd, n, O.TORUS, O.LIFE)
    with GolEngine(Wd, Hd) as e:
        assert e.pass_plan(n) == [10, 10]
        e.load(board)
        e.step(n)
        assert e.hash() == int(want[-1])
        assert np.array_equal(e.snapshot(), final)
        for gpp in (6, 7, 8, 9, 10, 11, 12):  # every wide multi-generation depth the planner may pick
            e.set_tuning(gens_per_pass=gpp)
            e.load(board)
            e.step(n)
            assert e.hash() == int(want[-1]), gpp


def _golden_262144():
    """The oracle's global hash of the seed-0x5EED 262144^2 torus at epochs
    0, 1, ... (tests/golden/bench_262144.json, tests/golden/make_bench_golden.py)."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bench_262144.json")
    with open(path) as f:
        return [int(x, 16) for x in json.load(f)["hashes"]]


def _oracle_rows(gens, lo, n):
    """Rows [lo, lo + n) of the seed-0x5EED 262144^2 torus after `gens`
    generations, from the oracle on their light cone alone: rows lo - gens ..
    lo + n + gens - 1 of the initial board (mod H), stepped `gens` times as a
    block whose ends wrap onto each other -- the wrong rows that brings in
    move one row per generation and never reach the middle n rows."""
    idx = [(lo - gens + k) % H for k in range(n + 2 * gens)]
    block = np.vstack([O.seed_packed(W, H, 0x5EED, row0=i, rows=1) for i in idx])
    out, _ = O.run_packed(block, W, gens, O.TORUS, O.LIFE, want_hashes=False)
    return out[gens:gens + n]


def test_config5_full_size_eight_shards_kill_3_at_25(gpu):
    """BASELINE.json configs[4] at its stated scale, on one GPU: the 262144^2
    torus as 8 in-process shards of 262144 x 32768 (the N = 8 decomposition),
    checkpoints every 10 generations in the background (gol_checkpoint_async),
    shard 3 killed at generation 25 of 50 and re-spawned alone from its last
    landed checkpoint and its neighbours' light cone (gol_replay), the other 7
    keeping their state (BoardCreator.scala:120-154, CellActor.scala:34,71-74).
    Every generation's global hash equals the oracle's (the committed golden
    table), the replayed partials complete the recorded global hashes
    (checked inside respawn), and the final board matches the oracle on rows
    around both of shard 3's seams and its middle."""
    from gameoflife import _native as N
    from gameoflife.fault import ShardedSimulation
    golden = _golden_262144()
    assert len(golden) > 50
    sim = ShardedSimulation(W, H, 8, list(range(N.device_count())), checkpoint_every=10, async_checkpoints=True)
    try:
        got = sim.run(50, crashes=[(25, 3)])
        assert got == golden[1:51]
        resp = [e for e in sim.events if e.startswith("respawn shard 3")]
        assert len(resp) == 1 and (resp[0].endswith("light cone 20->25") or resp[0].endswith("light cone 10->25"))
        assert sum(s.hash() for s in sim.shards) % (1 << 64) == golden[50]
        rows = H // 8
        snaps = {k: sim.shards[k].snapshot() for k in (2, 3, 4)}
        board = np.vstack([snaps[2][-64:], snaps[3], snaps[4][:64]])  # rows 3*rows - 64 .. 4*rows + 63
        base = 3 * rows - 64
        for lo in (3 * rows - 32, 3 * rows + rows // 2, 4 * rows - 32):
            np.testing.assert_array_equal(board[lo - base:lo - base + 64], _oracle_rows(50, lo, 64))
    finally:
        sim.close()

