"""GPU: the multi-rank ring schedule with several ranks on one GPU.

RCCL refuses two ranks on one GPU, so the pool's one-GPU box never runs
libgol's multi-rank exchange over RCCL ("the multi-rank RCCL
issue order is asserted only in Python").  gol_comm_init_loopback joins
contexts of one process -- one host thread each, as one process per GPU
would be -- into a ring whose transport executes exactly the halo operation
list one_pass hands to RCCL (gol_ring.cpp HaloOp: last rows -> down, first
rows -> up, top halo <- up, bottom halo <- down), matched per (sender,
receiver) pair in FIFO order like ncclSend / ncclRecv.  With N = 2 the up
and down peers coincide, so a wrong issue order swaps the halos.  Checked
bit-exact against the oracle (per-generation global hashes through the ring's
all-reduce, final boards), at full size against the golden table, and across
a ring rebuild (gol_comm_abort + re-init: config 5's survivors re-wiring,
BoardCreator.scala:129-130,138-154)."""
import json
import os
import threading
import uuid

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _ranks(W, H, world, topology="torus", gpp=0, seed=None, board=None):
    from gameoflife import _native as N
    from gameoflife.engine import GolEngine
    key = uuid.uuid4().hex
    engs = []
    for r in range(world):
        row0, rows = N.shard_rows(H, r, world)
        e = GolEngine(W, H, topology=topology, rule="life", row0=row0, rows=rows)
        e.set_tuning(gens_per_pass=gpp)
        if board is not None:
            e.load(board[row0:row0 + rows])
        else:
            e.seed(seed)
        e.comm_init_loopback(key, r, world)
        engs.append(e)
    return engs


def _run_threads(engs, fn):
    """fn(rank, engine) on one thread per rank; re-raises the first error."""
    out, errs = [None] * len(engs), []

    def work(r):
        try:
            out[r] = fn(r, engs[r])
        except Exception as exc:  # noqa: BLE001 -- reported to the test thread
            errs.append(exc)

    ts = [threading.Thread(target=work, args=(r,)) for r in range(len(engs))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(300)
    assert not any(t.is_alive() for t in ts), "a rank hung"
    if errs:
        raise errs[0]
    return out


def _step_global(engs, gens):
    """Every rank steps `gens` generations with fused hashes; the ring's
    all-reduce sums the shards' partials; returns the global hashes."""
    res = _run_threads(engs, lambda r, e: e.allreduce_u64(e.step(gens, hashes=True)))
    for h in res[1:]:
        np.testing.assert_array_equal(h, res[0])  # every rank got the same sums
    return res[0]


@pytest.mark.parametrize("world,topology,gpp", [(2, "torus", 1), (2, "torus", 4), (2, "torus", 12), (3, "torus", 0),
                                                (4, "torus", 6), (2, "ref-clipped", 3), (3, "ref-clipped", 0),
                                                (5, "torus", 0)])
def test_loopback_ring_matches_oracle(gpu, world, topology, gpp):
    from gameoflife import _native as N
    W, H, gens = 32 * 300 + (0 if topology == "torus" else 7), 97, 26
    topo = O.TORUS if topology == "torus" else O.REF_CLIPPED
    if topology == "torus":
        board = O.seed_packed(W, H, world * 31 + gpp)
    else:
        rng = np.random.default_rng(world)
        board = O.pack((rng.random((H, W)) < 0.5).astype(np.uint8))
    engs = _ranks(W, H, world, topology, gpp, board=board)
    try:
        N.take_hip_error()
        got = _step_global(engs, gens)
        final = np.vstack([e.snapshot() for e in engs])
        assert N.take_hip_error() == 0
    finally:
        for e in engs:
            e.close()
    final_cpu, want = O.run_packed(board, W, gens, topo, O.LIFE)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"first mismatch at generation {bad[0] + 1}"
    np.testing.assert_array_equal(final, final_cpu)


def test_loopback_two_ranks_deep_halos(gpu):
    """The N = 2 ring's up and down peers are the same rank: the halo each
    rank receives first must be its top one.  Checked against the oracle on
    a board whose top and bottom halos differ, at a depth that reads them."""
    W, H, gens = 32 * 64, 40, 12
    board = O.seed_packed(W, H, 4242)
    engs = _ranks(W, H, 2, gpp=12, board=board)
    try:
        got = _step_global(engs, gens)
        final = np.vstack([e.snapshot() for e in engs])
    finally:
        for e in engs:
            e.close()
    final_cpu, want = O.run_packed(board, W, gens, O.TORUS, O.LIFE)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(final, final_cpu)


def test_loopback_ring_rebuild(gpu):
    """3 ranks step, every rank leaves the ring (gol_comm_abort) and joins a
    new one, stepping on: bit-exact, no HIP status left pending."""
    from gameoflife import _native as N
    W, H = 32 * 200, 90
    board = O.seed_packed(W, H, 77)
    engs = _ranks(W, H, 3, board=board)
    try:
        h1 = _step_global(engs, 14)
        for e in engs:
            e.comm_abort()
        assert N.take_hip_error() == 0
        key = uuid.uuid4().hex
        for r, e in enumerate(engs):
            e.comm_init_loopback(key, r, 3)
        h2 = _step_global(engs, 14)
        assert N.take_hip_error() == 0
        final = np.vstack([e.snapshot() for e in engs])
    finally:
        for e in engs:
            e.close()
    final_cpu, want = O.run_packed(board, W, 28, O.TORUS, O.LIFE)
    np.testing.assert_array_equal(np.concatenate([h1, h2]), want)
    np.testing.assert_array_equal(final, final_cpu)


def test_loopback_full_size_eight_ranks_golden(gpu):
    """The driver's N = 8 decomposition of the bench board (262144^2, 8 ranks
    of 32768 rows; the bench's W + K = 5 + 20 unhashed generations, then 25
    with fused hashes, at the planner's passes) through the ring schedule's
    exact operation list, eight ranks on one GPU:
    the global hash after W + K = 25 generations and every hashed generation
    26..50 equal the oracle's golden table (tests/golden/bench_262144.json)."""
    W = H = 262144
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bench_262144.json")) as f:
        golden = [int(x, 16) for x in json.load(f)["hashes"]]
    engs = _ranks(W, H, 8, seed=0x5EED)
    try:
        def window(r, e):
            e.step(5)
            e.step(20)
            e.sync()
            return e.allreduce_u64(np.array([e.hash()], dtype=np.uint64))[0]
        h25 = _run_threads(engs, window)
        assert all(int(h) == golden[25] for h in h25)
        hs = _step_global(engs, 25)
        assert [int(x) for x in hs] == golden[26:51]
    finally:
        for e in engs:
            e.close()
