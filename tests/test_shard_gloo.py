"""Multi-rank path on CPU (world_size 2 and 3, gloo): row-block shards that
exchange halo rows exactly as libgol's RCCL ring does (gol_ring.cpp
one_pass: before every pass of G generations, the last G rows down and the
first G rows up, G-row halos back, in shard.HaloPlan's op order; the pass
depth capped at floor(H / N), shard.ring_depth_cap) and reduce per-generation
partial hashes must reproduce the unsharded board and hashes, on uneven
decompositions.  The compute here is the oracle (test double for the GPU):
each rank steps its rows plus both G-row halos G generations, and keeps its
own rows, which the garbage entering at the ends of the extended block (one
row per generation) never reaches.  What is under test is the
decomposition, the G-deep halo protocol and the hash reduction."""
import os
import socket

import numpy as np
import pytest

from gameoflife.shard import HaloPlan, combine_hashes, fixed_depth_plan, ring_depth_cap, shard_rows_py
from oracle import oracle as O

W, H, GENS = 32 * 9, 37, 13  # H = 37: uneven shards at N = 2 and 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _exchange(plan: HaloPlan, shard: np.ndarray, G: int):
    """Issue the plan's ops as gloo isend/irecv (one 'group'): messages of G
    rows, exactly the G * pitch slices libgol sends."""
    import torch
    import torch.distributed as dist
    reqs, recv = [], {}
    zero = np.zeros((G, shard.shape[1]), dtype=np.uint32)
    for kind, what, peer in plan.ops():
        if kind == "send":
            rows = shard[-G:] if what == "last" else shard[:G]
            reqs.append(dist.isend(torch.from_numpy(rows.astype(np.int32).copy()), peer))
        else:
            buf = torch.zeros((G, shard.shape[1]), dtype=torch.int32)
            reqs.append(dist.irecv(buf, peer))
            recv[what] = buf
    for r in reqs:
        r.wait()
    top = recv["top"].numpy().astype(np.uint32) if "top" in recv else zero
    bot = recv["bot"].numpy().astype(np.uint32) if "bot" in recv else zero
    return top, bot


def _worker(rank, world, port, torus, gpp, out_q):
    # torch is imported here, not at module level: the GPU session collects
    # this module too, and libgol must be the first to bind the HIP runtime
    # (tests/conftest.py)
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        row0, rows = shard_rows_py(H, rank, world)
        full = O.seed_packed(W, H, 1234)
        shard = full[row0:row0 + rows].copy()
        plan = HaloPlan(rank, world, torus)
        depths = fixed_depth_plan(GENS, ring_depth_cap(H, world, gpp))
        hashes = []
        for G in depths:
            assert G <= rows
            top, bot = _exchange(plan, shard, G)
            ext = np.vstack([top, shard, bot])  # ext row k = global row row0 - G + k
            for _ in range(G):
                if torus:
                    ext = O.step_packed(ext, W, O.TORUS, O.LIFE)
                else:
                    # clipped geometry, visible region = global [0,W-1) x [0,H-1)
                    ext = O.step_packed(ext, W, O.REF_CLIPPED, O.LIFE, vis=(W - 1, H - 1 - row0 + G))
                    if row0 == 0:
                        ext[:G] = 0  # global rows < 0 do not exist (the kernel reads them as dead)
                own = ext[G:G + rows]
                part = O.hash_packed(own, W, row0=row0, topology=O.TORUS if torus else O.REF_CLIPPED)
                t = torch.tensor([part - (1 << 64) if part >= (1 << 63) else part], dtype=torch.int64)
                dist.all_reduce(t)  # int64 sum wraps like uint64
                hashes.append(int(t.item()) & ((1 << 64) - 1))
            shard = ext[G:G + rows].copy()
        gathered = [None] * world
        dist.all_gather_object(gathered, (row0, shard.tolist()))
        if rank == 0:
            out_q.put((hashes, gathered, depths))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,torus,gpp", [(2, True, 1), (2, True, 8), (3, True, 6), (3, True, 8),
                                             (2, False, 3), (3, False, 8), (2, True, 12), (3, True, 12)])
def test_sharded_matches_unsharded(world, torus, gpp):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, torus, gpp, q), nprocs=world, start_method="spawn")
    hashes, gathered, depths = q.get(timeout=60)
    assert sum(depths) == GENS and max(depths) == min(gpp, H // world)
    board = np.vstack([np.array(s, dtype=np.uint32) for _, s in sorted(gathered)])
    topo = O.TORUS if torus else O.REF_CLIPPED
    ref, ref_h = O.run_packed(O.seed_packed(W, H, 1234), W, GENS, topo, O.LIFE)
    assert (board == ref).all()
    assert hashes == [int(x) for x in ref_h]


def test_halo_plan_two_ranks_pairs_rows_correctly():
    """With 2 ranks up == down; per-peer FIFO order must pair the sender's
    last row with the receiver's top halo."""
    p0, p1 = HaloPlan(0, 2, True), HaloPlan(1, 2, True)
    sends0 = [w for k, w, _ in p0.ops() if k == "send"]
    recvs1 = [w for k, w, _ in p1.ops() if k == "recv"]
    assert sends0 == ["last", "first"] and recvs1 == ["top", "bot"]
    # clipped: the ends of the ring do not wrap
    assert HaloPlan(0, 3, False).ops() == [("send", "last", 1), ("recv", "bot", 1)]
    assert HaloPlan(2, 3, False).ops() == [("send", "first", 1), ("recv", "top", 1)]


def test_combine_hashes_wraps_mod_2_64():
    a = np.array([2**64 - 1, 5], dtype=np.uint64)
    b = np.array([2, 7], dtype=np.uint64)
    assert combine_hashes([a, b]).tolist() == [1, 12]


def test_ring_depth_cap_mirrors_libgol():
    """floor(H / N) caps a ring's passes (every rank sends the same G rows);
    a 1-rank self-ring sends its own G rows, so G <= H."""
    assert ring_depth_cap(37, 3) == 12 and ring_depth_cap(37, 5) == 7 and ring_depth_cap(5, 1) == 5
    assert ring_depth_cap(262144, 8) == 12 and ring_depth_cap(262144, 8, 6) == 6
    assert ring_depth_cap(262144, 8, life_torus=False) == 8 and ring_depth_cap(262144, 8, 10, False) == 10
    assert fixed_depth_plan(13, 8) == [8, 5] and fixed_depth_plan(12, 6) == [6, 6]
