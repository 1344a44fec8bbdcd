"""Fault path: periodic shard checkpoints, shard loss and re-spawn.

Reference behaviour:
* a cell actor dies (node loss, or an injected ``DoCrashMsg``,
  ``BoardCreator.scala:97-102``, ``CellActor.scala:53-55,95-96``);
* ``BoardCreator.onCellTermination`` re-deploys it at the same position on a
  random surviving node with its epoch-0 state and re-wires the neighbour
  refs (``BoardCreator.scala:138-154``);
* the new cell replays epochs 1..step from its neighbours' never-pruned
  histories (``CellActor.scala:34,71-74,86``).

Here a shard (a row block in HBM) is the unit that dies.  Every
``checkpoint_every`` generations all shards save a consistent checkpoint
(``gol_checkpoint``: epoch + packed rows) to host memory (optionally also to
files).  When a shard is lost at epoch t, a new context for its rows is
created on a surviving GPU (possibly next to a shard it already hosts), it
restores its own checkpoint of epoch c, takes the t - c rows above and below
it at epoch c from its neighbours' checkpoints (the light cone) and replays
alone to epoch t (``gol_replay``, ``respawn``); the surviving shards keep
their state and wait, as the reference's surviving cells do.  Then the group
is rebuilt and the run continues.  (``respawn(..., mode="rollback")`` is the
older global rollback: every shard restores epoch c and the group replays.)
``run(generations, crashes)`` injects crashes on a schedule (``crash_schedule``
of the reference's errors.delay / errors.every / max-crashes keys).
Generations are a pure function of the checkpoint, so the per-generation
hashes equal those of an uninterrupted run.
"""
from __future__ import annotations

import os

import numpy as np

from .elastic import blob_rows, light_cone_from
from ._native import GolError
from .engine import GolEngine, ShardGroup, host_array
from .shard import shard_rows_py


class ShardedSimulation:
    def __init__(self, width: int, height: int, nshards: int, devices: list[int] | None = None,
                 topology: str = "torus", rule="life", seed: int = 0x5EED,
                 checkpoint_every: int = 10, checkpoint_dir: str | None = None,
                 gens_per_pass: int = 0, async_checkpoints: bool = False):
        self.width, self.height, self.n = width, height, nshards
        self.devices = list(devices) if devices else [0]
        self.topology, self.rule = topology, rule
        self.checkpoint_every = checkpoint_every
        self.checkpoint_dir = checkpoint_dir
        self.gens_per_pass = gens_per_pass
        # async_checkpoints: each checkpoint is taken in the background
        # (gol_checkpoint_async into page-locked buffers, two sets) while the
        # next generations run, and becomes the recovery point when it has
        # landed (the next checkpoint, a loss, a snapshot or close)
        self.async_checkpoints = async_checkpoints
        self._ckpt_bufs: list[list] = [[], []]
        self._ckpt_set = 0
        self._pending_epoch: int | None = None
        self.placement = [self.devices[k % len(self.devices)] for k in range(nshards)]
        self.shards: list[GolEngine | None] = [self._make(k, self.placement[k]) for k in range(nshards)]
        for s in self.shards:
            s.seed(seed)
        self.group: ShardGroup | None = ShardGroup(self.shards)
        self.hashes: list[int] = []          # global per-generation hashes, epochs 1..epoch
        self.partials: dict[int, list[int]] = {}  # epoch -> every shard's partial hash (since the last checkpoint)
        self.epoch = 0
        self.ckpt_epoch = -1
        self.ckpt: list[bytes] = []
        self.events: list[str] = []
        self.checkpoint()
        self._finish_checkpoint()  # epoch 0 is a recovery point before anything can be lost

    def _make(self, k: int, device: int) -> GolEngine:
        row0, rows = shard_rows_py(self.height, k, self.n)
        e = GolEngine(self.width, self.height, topology=self.topology, rule=self.rule, device=device,
                      row0=row0, rows=rows)
        e.set_tuning(gens_per_pass=self.gens_per_pass)
        return e

    # ----------------------------------------------------------- checkpoints
    def checkpoint(self) -> None:
        if self.async_checkpoints:
            self._finish_checkpoint()
            bufs = self._ckpt_bufs[self._ckpt_set]
            if not bufs:
                bufs.extend(host_array((s.checkpoint_bytes(),), np.uint8) for s in self.shards)
            for s, b in zip(self.shards, bufs):
                s.checkpoint_async(b)
            self._pending_epoch = self.epoch
            return
        self._commit_checkpoint([s.checkpoint() for s in self.shards], self.epoch)

    def _finish_checkpoint(self) -> None:
        """Wait for a background checkpoint and make it the recovery point."""
        if self._pending_epoch is None:
            return
        for s in self.shards:
            s.snapshot_wait()
        blobs = self._ckpt_bufs[self._ckpt_set]
        self._ckpt_set ^= 1  # the next one goes to the other set; this one stays valid
        epoch, self._pending_epoch = self._pending_epoch, None
        self._commit_checkpoint(list(blobs), epoch)

    def _drop_checkpoint(self, lost: int, landed: bool | None = None) -> None:
        """Shard `lost` dies while a background checkpoint may be in flight.
        If its part has reached host memory (gol_snapshot_query; `landed`
        forces the answer) the set is complete and is committed; otherwise
        that part never lands, so the set is discarded (the survivors' copies
        are waited for, to release their buffers) and the previous committed
        checkpoint stays the recovery point."""
        if self._pending_epoch is None:
            return
        if landed is None:
            # On a truly lost device the query itself fails: a checkpoint
            # whose landing cannot be confirmed never existed.
            try:
                landed = self.shards[lost].snapshot_landed()
            except GolError:
                landed = False
        if landed:
            self._finish_checkpoint()
            return
        for j, s in enumerate(self.shards):
            if j != lost:
                s.snapshot_wait()
        self.events.append(f"checkpoint@{self._pending_epoch} dropped (shard {lost} lost in flight)")
        self._pending_epoch = None  # the set is rewritten by the next checkpoint

    def _commit_checkpoint(self, blobs: list, epoch: int) -> None:
        self.ckpt = blobs
        self.ckpt_epoch = epoch
        self.partials = {e: p for e, p in self.partials.items() if e > epoch}
        if self.checkpoint_dir:
            os.makedirs(self.checkpoint_dir, exist_ok=True)
            for k, blob in enumerate(self.ckpt):
                tmp = os.path.join(self.checkpoint_dir, f"shard{k}.ckpt.tmp")
                with open(tmp, "wb") as f:
                    f.write(blob)
                os.replace(tmp, os.path.join(self.checkpoint_dir, f"shard{k}.ckpt"))
        self.events.append(f"checkpoint@{epoch}")

    # ------------------------------------------------------------------ run
    def step(self, generations: int) -> list[int]:
        """Advance, checkpointing at every multiple of checkpoint_every."""
        if self.group is None:
            raise RuntimeError("a shard is lost: respawn() before stepping")
        out: list[int] = []
        while generations > 0:
            k = self.checkpoint_every
            to_ckpt = (k - self.epoch % k) if k else generations
            n = min(generations, to_ckpt)
            glob, part = self.group.step(n, partials=True)
            hs = [int(h) for h in glob]
            for g in range(n):
                self.partials[self.epoch + g + 1] = [int(x) for x in part[:, g]]
            self.epoch += n
            self.hashes.extend(hs)
            out.extend(hs)
            generations -= n
            if k and self.epoch % k == 0:
                self.checkpoint()
        return out

    # ---------------------------------------------------------------- faults
    def kill(self, k: int, checkpoint_landed: bool | None = None) -> None:
        """Lose shard k (its context and device memory are gone).  A
        background checkpoint still in flight on shard k is lost with it
        (checkpoint_landed: force whether it had landed; None asks the
        device)."""
        self._drop_checkpoint(k, checkpoint_landed)
        self.shards[k].close()            # the group now has a hole (gol_group_step -> GOL_ESTATE)
        self.shards[k] = None
        self.group.close()
        self.group = None
        self.events.append(f"kill shard {k} @{self.epoch}")

    def _checkpoint_blobs(self) -> list[bytes]:
        if not self.checkpoint_dir:
            return self.ckpt
        blobs = []  # survive the loss of host memory too
        for j in range(self.n):
            with open(os.path.join(self.checkpoint_dir, f"shard{j}.ckpt"), "rb") as f:
                blobs.append(f.read())
        return blobs

    def respawn(self, k: int, device: int | None = None, mode: str = "light-cone") -> list[int]:
        """Re-spawn shard k on `device` (default: the next surviving device).

        light-cone: shard k restores its checkpoint (epoch c) and replays the
        lost generations c+1..epoch alone from its neighbours' checkpoint rows
        (gol_replay); the other shards keep their state.  Returns shard k's
        replayed per-generation partial hashes.
        rollback: every shard restores epoch c and the group replays; returns
        the replayed global hashes, checked against the lost ones."""
        if device is None:
            alive = [d for d in self.devices if d != self.placement[k]] or self.devices
            device = alive[0]
        self.placement[k] = device
        self.shards[k] = self._make(k, device)
        blobs = self._checkpoint_blobs()
        if mode == "rollback":
            for s, blob in zip(self.shards, blobs):
                s.restore(blob)
            target = self.epoch
            self.epoch = self.ckpt_epoch
            lost = self.hashes[self.ckpt_epoch:]
            del self.hashes[self.ckpt_epoch:]
            self.group = ShardGroup(self.shards)
            self.events.append(f"respawn shard {k} on device {device}, rollback to {self.ckpt_epoch}")
            replayed = self.step(target - self.epoch) if target > self.epoch else []
            if replayed != lost:
                raise AssertionError("replayed generations differ from the lost ones")
            return replayed
        s = self.shards[k]
        s.restore(blobs[k])
        d = self.epoch - self.ckpt_epoch
        up, dn = light_cone_from(lambda idx: blob_rows(blobs, idx), s.row0, s.rows, d, self.height,
                                 self.topology == "torus", s.wwords)
        part = [int(h) for h in s.replay(d, up, dn)] if d else []
        # the replayed partials must complete the global hashes recorded
        # before the loss: survivors' partials + shard k's == global, mod 2^64
        for g, p in enumerate(part, start=self.ckpt_epoch + 1):
            others = sum(v for j, v in enumerate(self.partials[g]) if j != k)
            if (others + p) % (1 << 64) != self.hashes[g - 1]:
                raise AssertionError(f"replayed partial of shard {k} at generation {g} does not complete "
                                     "the recorded global hash")
            self.partials[g][k] = p
        self.group = ShardGroup(self.shards)
        self.events.append(f"respawn shard {k} on device {device}, light cone {self.ckpt_epoch}->{self.epoch}")
        return part

    def run(self, generations: int, crashes: list[tuple[int, int]] = ()) -> list[int]:
        """Advance `generations`, crashing shard pick % n after each crash
        generation (board.crash_schedule) and re-spawning it alone."""
        out: list[int] = []
        end = self.epoch + generations
        for g, pick in sorted(crashes):
            if g <= self.epoch or g > end:
                continue
            out.extend(self.step(g - self.epoch))
            k = pick % self.n
            self.kill(k)
            self.respawn(k)
        out.extend(self.step(end - self.epoch))
        return out

    def snapshot(self) -> np.ndarray:
        self._finish_checkpoint()
        return np.vstack([s.snapshot() for s in self.shards])

    def close(self) -> None:
        if all(s is not None for s in self.shards):
            self._finish_checkpoint()
        if self.group is not None:
            self.group.close()
        for s in self.shards:
            if s is not None:
                s.close()
