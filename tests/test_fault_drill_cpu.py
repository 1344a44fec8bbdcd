"""CPU: the multi-GPU bench's fault drill (gameoflife.elastic.ring_fault_drill)
with its ranks as threads and an oracle-backed engine double.

The double's board is the oracle's truth table (tests only: it imports
oracle/); its all-reduce is a barrier over the ranks' threads.  restore()
accepts a blob only if it holds exactly the truth rows of its block at its
epoch, and replay() steps the block plus the light cone it is handed with the
oracle -- so the drill's checkpoint bookkeeping (which files exist, which
epoch it recovers from, which rows it reads) is checked, not only its control
flow.  The loss epoch covers both cases of BoardCreator.scala:120-154's
re-deploy: between two checkpoints (kill_at = 25, every = 10) and ON a
checkpoint epoch (kill_at % every == 0), where the lost rank dies before it
writes that epoch's file and its neighbours must keep their previous one."""
import os
import threading

import numpy as np
import pytest

from oracle import oracle as O

M64 = (1 << 64) - 1


class _Ring:
    """All-reduce (sum mod 2^64) over `world` threads."""

    def __init__(self, world):
        self.world = world
        self.bar = threading.Barrier(world, timeout=60)
        self.slots = [None] * world
        self.out = None

    def allreduce(self, rank, values):
        v = [int(x) for x in np.asarray(values, dtype=np.uint64)]
        self.slots[rank] = v
        if self.bar.wait() == 0:
            self.out = [sum(col) & M64 for col in zip(*self.slots)]
        self.bar.wait()
        out = np.array(self.out, dtype=np.uint64)
        self.bar.wait()
        return out


class _Truth:
    def __init__(self, W, H, seed, gens):
        self.W, self.H = W, H
        b = O.seed_packed(W, H, seed)
        self.boards = [b]
        for _ in range(gens + 1):
            b, _ = O.run_packed(b, W, 1, O.TORUS, O.LIFE, want_hashes=False)
            self.boards.append(b)

    def rows(self, e, r0, n):
        return self.boards[e][np.arange(r0, r0 + n) % self.H]


class _Engine:
    def __init__(self, truth, row0, rows):
        self.t, self.row0, self.rows, self.epoch = truth, row0, rows, 0
        self.ring, self.rank = None, None

    def _mine(self, e=None):
        return self.t.rows(self.epoch if e is None else e, self.row0, self.rows)

    def seed(self, seed):
        self.epoch = 0

    def _part(self, e):
        return O.hash_packed(self._mine(e), self.t.W, row0=self.row0)

    def step(self, n, hashes=False):
        e0 = self.epoch
        self.epoch += n
        return np.array([self._part(e0 + k + 1) for k in range(n)], dtype=np.uint64) if hashes else None

    def hash(self):
        return self._part(self.epoch)

    def allreduce_u64(self, values):
        return self.ring.allreduce(self.rank, values)

    def checkpoint(self):
        from gameoflife.elastic import make_checkpoint
        return make_checkpoint(dict(width=self.t.W, height=self.t.H, row0=self.row0, epoch=self.epoch, topology=0,
                                    birth=8, survive=12), self._mine())

    def restore(self, blob):
        from gameoflife.elastic import parse_checkpoint
        h, data = parse_checkpoint(bytes(blob))
        assert (h["row0"], h["rows"]) == (self.row0, self.rows)
        np.testing.assert_array_equal(data, self._mine(h["epoch"]))
        self.epoch = h["epoch"]

    def replay(self, d, above, below):
        ext = np.vstack([above, self._mine(), below]).astype(np.uint32)
        hs = []
        for _ in range(d):
            ext = O.step_packed(ext, self.t.W, O.TORUS, O.LIFE)
            self.epoch += 1
            blk = ext[d:d + self.rows]
            hs.append(O.hash_packed(blk, self.t.W, row0=self.row0))
        np.testing.assert_array_equal(ext[d:d + self.rows], self._mine())  # the light cone was the right one
        return np.array(hs, dtype=np.uint64)

    def snapshot(self, out=None):
        d = self._mine()
        if out is None:
            return d.copy()
        out[...] = d
        return out

    def comm_abort(self):
        self.ring = None

    def close(self):
        pass


def _run(tmp_path, world, victim, kill_at, every, gens=50, W=256, H=64, seed=0x5EED):
    from gameoflife.elastic import ring_fault_drill
    from gameoflife.shard import shard_rows_py
    truth = _Truth(W, H, seed, gens)
    rings = {"first": _Ring(world), "fault": _Ring(world - 1)}
    make = lambda r0, n: _Engine(truth, r0, n)  # noqa: E731

    def join(e, tag, r, w):
        assert rings[tag].world == w
        e.ring, e.rank = rings[tag], r

    engs = []
    for r in range(world):
        e = make(*shard_rows_py(H, r, world))
        join(e, "first", r, world)
        engs.append(e)
    out, errs = [None] * world, []

    def work(r):
        try:
            out[r] = ring_fault_drill(engs[r], make, join, r, world, W, H, str(tmp_path), seed=seed, victim=victim,
                                      kill_at=kill_at, gens=gens, every=every)
        except Exception as exc:  # noqa: BLE001 -- reported to the test thread
            errs.append(exc)
            for g in rings.values():
                g.bar.abort()

    ts = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert not any(t.is_alive() for t in ts), "a rank hung"
    if errs:
        raise errs[0]
    want = [int(O.hash_packed(truth.boards[e], W)) for e in range(gens + 1)]
    return out, want


@pytest.mark.parametrize("world,victim,kill_at,every", [
    (4, 3, 25, 10),   # the bench's drill: lost between checkpoints
    (4, 3, 30, 10),   # lost ON a checkpoint epoch: it never writes 30, the others keep 20
    (4, 0, 20, 10),
    (3, 1, 10, 10),   # lost at the first checkpoint epoch: no earlier file to recover from
    (2, 1, 40, 20),
])
def test_ring_fault_drill_recovers(tmp_path, world, victim, kill_at, every):
    if kill_at == every:
        # No checkpoint precedes the first one, so a loss at the first
        # checkpoint epoch has nothing to recover from: the drill must say so.
        with pytest.raises(FileNotFoundError):
            _run(tmp_path, world, victim, kill_at, every)
        return
    out, want = _run(tmp_path, world, victim, kill_at, every)
    lost = [r for r, (e, _) in enumerate(out) if e is None]
    assert lost == [victim]
    c_expect = (kill_at - 1) // every * every  # the victim's last own checkpoint
    for e, rep in out:
        if e is None:
            continue
        c = rep["checkpoint_epoch"]
        assert c == c_expect
        assert rep["before"] == want[1:kill_at + 1]
        assert rep["replayed"] == want[c + 1:kill_at + 1]
        assert rep["at_recovery"] == want[kill_at]
        assert rep["after"] == want[kill_at + 1:51]
        assert rep["final"] == want[50]


def test_checkpoint_files_pruned_once_complete(tmp_path):
    """Only complete epochs let a rank drop its previous file: after a loss
    between checkpoints the directory holds just the last complete epoch."""
    from gameoflife.elastic import complete_epochs, epoch_dir
    _run(tmp_path, 4, 3, 25, 10)
    assert complete_epochs(str(tmp_path), 64) == [20]
    files = {d: len(os.listdir(os.path.join(str(tmp_path), d))) for d in os.listdir(str(tmp_path))}
    assert {d: n for d, n in files.items() if n} == {os.path.basename(epoch_dir(str(tmp_path), 20)): 4}
