"""Row-block sharding over GPUs (one backend process per GPU).

The reference scales by adding backend JVMs and deploying cell actors on a
random node (BoardCreator.scala:33-36,65-70); neighbours then talk across the
network (application.conf:11-17).  Here rank r of n owns the contiguous row
block ``gol_shard_rows(H, r, n)``.  Before every pass of G generations it
exchanges G halo rows with each ring neighbour over RCCL (inside libgol,
gol_ring.cpp one_pass): its first G rows go up, its last G rows go down, and
G-row halos come back.  This module holds the host-side pieces: the halo plan
(the exact op order and message shapes libgol issues, shared with the CPU
tests), the pass-depth cap, the hash reduction and the per-process backend
worker.
"""
from __future__ import annotations

import dataclasses

import numpy as np


def shard_rows_py(height: int, rank: int, nranks: int) -> tuple[int, int]:
    """Pure-Python twin of gol_shard_rows (contiguous blocks, the first
    height % nranks ranks one row longer)."""
    if height <= 0 or nranks <= 0 or not 0 <= rank < nranks or height < nranks:
        raise ValueError("bad shard arguments")
    base, extra = divmod(height, nranks)
    return rank * base + min(rank, extra), base + (1 if rank < extra else 0)


MAX_GENS_PER_PASS = 12  # gol_kernels.h kMaxGensPerPass
MAX_GENS_PLANNED_GENERIC = 8  # gol_schedule.cpp kMaxGensPlannedGeneric


def ring_depth_cap(height: int, nranks: int, gens_per_pass: int = 0, life_torus: bool = True) -> int:
    """Deepest pass a ring may run (gol_schedule.cpp depth_cap): every rank must
    issue identical halo messages, so the depth is capped by the smallest
    shard, floor(H / N) rows (a 1-rank self-ring: H).  Planned passes of
    other rules / the clipped topology stop at 8."""
    g = gens_per_pass if gens_per_pass > 0 else (MAX_GENS_PER_PASS if life_torus else MAX_GENS_PLANNED_GENERIC)
    return max(1, min(g, MAX_GENS_PER_PASS, height // nranks))


def fixed_depth_plan(generations: int, depth: int) -> list[int]:
    """Pass depths of a fixed gens_per_pass (gol_schedule.cpp plan_passes: taken
    literally, the last pass shorter)."""
    plan, done = [], 0
    while done < generations:
        plan.append(min(depth, generations - done))
        done += plan[-1]
    return plan


@dataclasses.dataclass(frozen=True)
class HaloPlan:
    """Halo exchange of one rank before each pass (gol_ring.cpp one_pass).

    A pass of G generations sends the rank's last G rows down and its first G
    rows up, and receives the G rows above it (top halo) and below it (bottom
    halo).  ops are issued inside one group in this order; with 2 ranks (or 1,
    the self-ring) up == down and per-peer FIFO matching pairs the sender's
    last rows with the receiver's top halo and its first rows with the bottom
    halo."""
    rank: int
    nranks: int
    torus: bool

    @property
    def up(self) -> int:
        return (self.rank + self.nranks - 1) % self.nranks

    @property
    def down(self) -> int:
        return (self.rank + 1) % self.nranks

    @property
    def has_up(self) -> bool:
        return self.torus or self.rank > 0

    @property
    def has_down(self) -> bool:
        return self.torus or self.rank < self.nranks - 1

    def ops(self) -> list[tuple[str, str, int]]:
        out = []
        if self.has_down:
            out.append(("send", "last", self.down))
        if self.has_up:
            out.append(("send", "first", self.up))
        if self.has_up:
            out.append(("recv", "top", self.up))
        if self.has_down:
            out.append(("recv", "bot", self.down))
        return out


def combine_hashes(partials: list[np.ndarray]) -> np.ndarray:
    """Global per-generation hash = sum of the shards' partials mod 2^64."""
    acc = np.zeros_like(np.asarray(partials[0], dtype=np.uint64))
    with np.errstate(over="ignore"):
        for p in partials:
            acc = acc + np.asarray(p, dtype=np.uint64)
    return acc


class BackendWorker:
    """One backend per GPU: owns its row block, joins
    the RCCL ring and advances in lockstep with the other ranks.

    ``control`` is the host control plane used only for the communicator id
    broadcast and the per-generation hash reduction (torch.distributed gloo
    in bench.py; any object with ``broadcast_bytes(b, root)``)."""

    def __init__(self, width: int, height: int, rank: int, nranks: int, device: int,
                 topology: str = "torus", rule="life", control=None):
        from . import _native as N
        from .engine import GolEngine
        self.rank, self.nranks = rank, nranks
        self.row0, self.rows = N.shard_rows(height, rank, nranks)
        self.engine = GolEngine(width, height, topology=topology, rule=rule, device=device,
                                row0=self.row0, rows=self.rows)
        if nranks > 1:
            if control is None:
                raise ValueError("a control plane is needed for nranks > 1")
            uid = N.unique_id() if rank == 0 else bytes(N.GOL_UNIQUE_ID_BYTES)
            uid = control.broadcast_bytes(uid, 0)
            self.engine.comm_init(uid, rank, nranks)

    def step(self, generations: int, hashes: bool = False):
        part = self.engine.step(generations, hashes=hashes)
        if not hashes:
            return None
        if self.nranks > 1:
            return self.engine.allreduce_u64(part)
        return part

    def close(self) -> None:
        self.engine.close()
