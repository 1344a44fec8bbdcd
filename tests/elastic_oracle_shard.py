"""CPU test double of gameoflife.elastic.GpuShard (torus, any rule mask):
the shard steps with the oracle, halo rows and the hash reduction go over
gloo, and the light-cone replay of a lost block is the oracle stepping the
block plus its light cone.  Lets the CPU suite run the elastic supervisor /
worker processes end to end.  Test infrastructure only (imports oracle/)."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gameoflife.elastic import make_checkpoint, parse_checkpoint  # noqa: E402
from gameoflife.rules import rule_by_name  # noqa: E402
from gameoflife.shard import HaloPlan  # noqa: E402
from oracle import oracle as O  # noqa: E402


class OracleShard:
    def __init__(self, width, height, row0, rows, topology="torus", rule="life", device=0):
        assert topology == "torus"
        self.W, self.H, self.row0, self.rows = width, height, row0, rows
        r = rule_by_name(rule)
        self.rule = (r.birth, r.survive)
        self.world, self.epoch = 1, 0
        self.plan = HaloPlan(0, 1, True)
        self.board = None

    def join(self, ring_dir, rank, world):
        self.world = world
        self.plan = HaloPlan(rank, world, True)
        if world > 1:
            dist.init_process_group("gloo", init_method="file://" + os.path.join(ring_dir, "gloo_store"),
                                    rank=rank, world_size=world)

    def leave(self):
        if dist.is_initialized():
            dist.destroy_process_group()
        self.world = 1

    def seed(self, seed):
        self.board = O.seed_packed(self.W, self.H, seed, row0=self.row0, rows=self.rows)
        self.epoch = 0

    def restore(self, blob):
        h, data = parse_checkpoint(blob)
        assert (h["row0"], h["rows"]) == (self.row0, self.rows)
        self.board, self.epoch = data.copy(), h["epoch"]

    def checkpoint(self):
        return make_checkpoint(dict(width=self.W, height=self.H, row0=self.row0, epoch=self.epoch,
                                    topology=0, birth=self.rule[0], survive=self.rule[1]), self.board)

    def _halos(self):
        if self.world == 1:
            return self.board[-1], self.board[0]
        reqs, recv = [], {}
        for kind, what, peer in self.plan.ops():
            if kind == "send":
                row = self.board[-1] if what == "last" else self.board[0]
                reqs.append(dist.isend(torch.from_numpy(row.view(np.int32).copy()), peer))
            else:
                recv[what] = torch.zeros(self.board.shape[1], dtype=torch.int32)
                reqs.append(dist.irecv(recv[what], peer))
        for q in reqs:
            q.wait()
        return recv["top"].numpy().view(np.uint32), recv["bot"].numpy().view(np.uint32)

    def step(self, n):
        glob, part = [], []
        for _ in range(n):
            top, bot = self._halos()
            ext = np.vstack([top[None], self.board, bot[None]])
            self.board = O.step_packed(ext, self.W, O.TORUS, self.rule)[1:-1]
            self.epoch += 1
            p = O.hash_packed(self.board, self.W, row0=self.row0)
            part.append(p)
            if self.world > 1:
                t = torch.tensor([p - (1 << 64) if p >= (1 << 63) else p], dtype=torch.int64)
                dist.all_reduce(t)  # int64 sum wraps like uint64
                p = int(t.item()) & ((1 << 64) - 1)
            glob.append(p)
        return np.array(glob, dtype=np.uint64), np.array(part, dtype=np.uint64)

    def close(self):
        self.leave()

    @staticmethod
    def replay_block(width, height, blob, above, below, depth, topology="torus", rule="life", device=0):
        r = rule_by_name(rule)
        h, data = parse_checkpoint(blob)
        ext = np.vstack([above, data, below]).astype(np.uint32)
        hs = []
        for _ in range(depth):
            ext = O.step_packed(ext, width, O.TORUS, (r.birth, r.survive))
            hs.append(O.hash_packed(ext[depth:depth + h["rows"]], width, row0=h["row0"]))
        return ext[depth:depth + h["rows"]].copy(), np.array(hs, dtype=np.uint64)
