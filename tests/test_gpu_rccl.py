"""GPU: the RCCL-sharded path (gol_comm_init + G-deep halo send/recv) with
2 and 3 ranks, one process each, all on the box's GPU(s).  If RCCL refuses
several ranks on one GPU (duplicate-GPU check) and the box has fewer GPUs
than ranks, the test is skipped with RCCL's message -- the driver's
multi-GPU bench then exercises the path."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

W, H, GENS = 32 * 300, 96, 14


def _worker(rank, world, uid_q, out_q, topology, gpp):
    try:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        from gameoflife import _native as N
        from gameoflife.engine import GolEngine
        ndev = N.device_count()
        row0, rows = N.shard_rows(H, rank, world)
        e = GolEngine(W, H, topology=topology, rule="life", device=rank % ndev, row0=row0, rows=rows)
        e.set_tuning(gens_per_pass=gpp)
        full = O.seed_packed(W, H, 99)
        e.load(full[row0:row0 + rows])
        if rank == 0:
            uid = N.unique_id()
            for _ in range(world - 1):
                uid_q.put(uid)
        else:
            uid = uid_q.get(timeout=60)
        e.comm_init(uid, rank, world)
        part = e.step(GENS, hashes=True)
        total = e.allreduce_u64(part)
        out_q.put((rank, row0, e.snapshot(), total.tolist(), None))
        e.close()
    except Exception as exc:  # report instead of hanging the parent
        out_q.put((rank, None, None, None, f"{type(exc).__name__}: {exc}"))


@pytest.mark.parametrize("world,topology,gpp", [(2, "torus", 1), (2, "torus", 6), (3, "torus", 4),
                                                (2, "ref-clipped", 3)])
def test_rccl_ring_matches_oracle(gpu, world, topology, gpp):
    ctx = mp.get_context("spawn")
    uid_q, out_q = ctx.Queue(), ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, uid_q, out_q, topology, gpp)) for r in range(world)]
    for p in procs:
        p.start()
    res = []
    try:
        for _ in range(world):
            res.append(out_q.get(timeout=180))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = [r[4] for r in res if r[4]]
    if errs:
        from gameoflife import _native as N
        if N.device_count() < world and any("duplicate" in e.lower() or "rccl" in e.lower()
                                            or "ncclInvalidUsage" in e for e in errs):
            pytest.skip(f"RCCL cannot place {world} ranks on {N.device_count()} GPU(s): {errs[0]}")
        raise AssertionError(errs)
    res.sort()
    board = np.vstack([r[2] for r in res])
    topo = O.TORUS if topology == "torus" else O.REF_CLIPPED
    ref, want = O.run_packed(O.seed_packed(W, H, 99), W, GENS, topo, O.LIFE)
    for r in res:
        assert r[3] == [int(x) for x in want]
    assert (board == ref).all()


# --------------------------------------------------------------------------
# 1-rank self-ring: the RCCL ring schedule on the box's single GPU.  A context
# with a 1-rank communicator runs gol_ring.cpp one_pass's sharded branch
# (interior rows || ncclSend/ncclRecv of G rows to itself, then the boundary
# rows on the edge stream after the exchange event), so every depth and the
# rows <= 2G path are checked against the oracle here, not only in the
# driver's multi-GPU bench.

@pytest.mark.parametrize("Hs,gpp,hashed", [(97, 1, True), (203, 6, True), (203, 8, True), (203, 8, False),
                                           (203, 0, True), (203, 0, False), (12, 8, True), (5, 8, True),
                                           (301, 3, False), (203, 12, True), (203, 10, False), (12, 12, True)])
def test_rccl_self_ring_matches_oracle(gpu, Hs, gpp, hashed):
    from gameoflife import _native as N
    from gameoflife.engine import GolEngine
    Ws, gens = 32 * 300, 23
    board = O.seed_packed(Ws, Hs, 1000 + Hs)
    final, want = O.run_packed(board, Ws, gens, O.TORUS, O.LIFE)
    with GolEngine(Ws, Hs) as e:
        e.set_tuning(gens_per_pass=gpp)
        e.load(board)
        e.comm_init(N.unique_id(), 0, 1)
        plan = e.pass_plan(gens, hashes=hashed)
        assert max(plan) <= min(12, Hs) and sum(plan) == gens
        got = e.step(gens, hashes=hashed)
        if hashed:
            np.testing.assert_array_equal(e.allreduce_u64(got), want)
        assert e.hash() == int(want[-1])
        assert np.array_equal(e.snapshot(), final)
        assert e.epoch == gens


def test_rccl_self_ring_clipped_and_rule(gpu):
    """A clipped board has no ring neighbours (dead rows above and below):
    the 1-rank ring schedule still runs interior + boundary launches."""
    from gameoflife import _native as N
    from gameoflife.engine import GolEngine
    Wc, Hc, gens = 32 * 40 + 7, 61, 17
    board = O.seed_packed(Wc, Hc, 3)
    final, want = O.run_packed(board, Wc, gens, O.REF_CLIPPED, O.LIFE)
    with GolEngine(Wc, Hc, topology="ref-clipped", rule="life") as e:
        e.load(board)
        e.comm_init(N.unique_id(), 0, 1)
        np.testing.assert_array_equal(e.step(gens, hashes=True), want)
        assert np.array_equal(e.snapshot(), final)
