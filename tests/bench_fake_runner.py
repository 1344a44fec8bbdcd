"""Runs bench.py's main() with a stand-in for libgol (test infrastructure for
tests/test_bench_multirank.py, not a test module).

The N > 1 control flow of bench.py -- the communicator id passed through the
rendezvous file, barriers, the settle loop, max-over-ranks time, the per-rank
diagnostics gathered over the ring, the per-rank 65536^2 run, the one JSON
line on rank 0 -- only runs for real on the driver's multi-GPU node.  This
runner replaces the native engine by a recorder so that flow can run on CPU
ranks: every engine call is appended to $FAKE_LOG_DIR/rank<r>.log, and the
engine's all-reduce (gol_comm_allreduce_u64 over RCCL in bench.py) runs over
a gloo process group the runner creates -- bench.py itself imports no torch.

    RANK=.. WORLD_SIZE=.. MASTER_ADDR=127.0.0.1 MASTER_PORT=.. FAKE_LOG_DIR=.. \
        python tests/bench_fake_runner.py --gpus N --steps K --warmup W ...
"""
import json
import os
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RANK = int(os.environ.get("RANK", "0"))
LOG = os.path.join(os.environ["FAKE_LOG_DIR"], f"rank{RANK}.log")


def log(*parts):
    with open(LOG, "a") as f:
        f.write(" ".join(str(p) for p in parts) + "\n")


M64 = (1 << 64) - 1


def golden(width, height):
    if (width, height) == (4096, 4096):  # configs[1]'s table lives in golden.json
        with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
            ent = next(e for e in json.load(f)["torus"] if (e["W"], e["H"], e["seed"]) == (4096, 4096, 0x5EED))
        return [int(ent["hash0"])] + [int(h) for h in ent["hashes"]]
    name = f"bench_{width}.json" if width == height else f"bench_{width}x{height}.json"
    with open(os.path.join(ROOT, "tests", "golden", name)) as f:
        return [int(x, 16) for x in json.load(f)["hashes"]]


def _mix(x):
    """splitmix64's finaliser on a uint64 array (wraps mod 2^64)."""
    with np.errstate(over="ignore"):
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


class FakeBoard:
    """A W x Hb torus whose "cells" are one u64 per row, c(y, e) at epoch e:
    pseudo-random for y > 0, and row 0 carries the rest of the golden hash of
    epoch e -- so the sum over any decomposition of the rows is the golden
    value, and only the whole sum is (a partial sum is a meaningless share).
    A row's data is its u64 as two u32 words (wwords = 2)."""

    _rest = {}

    def __init__(self, width, hb):
        self.w, self.hb = width, hb
        self.table = golden(width, hb)

    def rows(self, ys, e):
        ys = np.asarray(ys, dtype=np.int64) % self.hb
        with np.errstate(over="ignore"):
            v = _mix(ys.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15) + np.uint64(e + 1) * np.uint64(0xD1B54A32D192ED03)
                     + np.uint64(self.hb))
        if (ys == 0).any():
            key = (self.w, self.hb, e)
            if key not in self._rest:
                with np.errstate(over="ignore"):
                    rest = int(_mix(np.arange(1, self.hb, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
                                    + np.uint64(e + 1) * np.uint64(0xD1B54A32D192ED03) + np.uint64(self.hb)).sum())
                self._rest[key] = rest & M64
            g = self.table[e] if e < len(self.table) else 0
            v[ys == 0] = np.uint64((g - self._rest[key]) & M64)
        return v

    def block_sum(self, row0, rows, e):
        with np.errstate(over="ignore"):
            return int(self.rows(np.arange(row0, row0 + rows), e).sum()) & M64

    @staticmethod
    def words(v):
        return np.stack([(v & np.uint64(0xFFFFFFFF)).astype(np.uint32), (v >> np.uint64(32)).astype(np.uint32)], axis=1)


class FakeEngine:
    """Records calls; its state is a block of FakeBoard rows at an epoch: the
    state hash is the block's sum (so only the sum over all ranks -- the
    all-reduce -- equals the golden value), checkpoints / snapshots carry the
    rows' words, restore checks that a blob holds exactly the rows of its
    block at its epoch, and replay checks the light cone it is handed -- so
    the fault drill's bookkeeping (which rows, which epoch, merged in which
    order) is checked, not just its control flow."""

    wwords = 2

    def __init__(self, width, height, topology="torus", rule="life", device=0, row0=0, rows=0):
        self.w, self.h, self.row0, self.rows = width, height, row0, rows or height
        self.gens = self.launches = 0
        self.ms = 0.0
        self.epoch = 0
        self.whole = self.rows == height
        world = int(os.environ.get("WORLD_SIZE", "1"))
        # in a multi-rank job a shard is rows of the global torus; alone, a
        # context with fewer rows is a torus of its own height (as libgol's)
        self.board = FakeBoard(width, height if world > 1 else self.rows) if topology == "torus" else None
        if world == 1:
            self.row0 = 0
        self.corrupt = os.environ.get("FAKE_CORRUPT_RANK") == str(RANK)
        # the reference's default 7 x 7 board (bench.py default_board_run):
        # its per-generation hashes come from golden.json's ref_default entry
        self.ref_default = None
        if topology == "ref-clipped":
            with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
                ent = next(e for e in json.load(f)["ref_default"] if e["java_seed"] == 42)
            self.ref_default = [int(h) for h in ent["modes"][rule]["hashes"]]
        log("create", f"{width}x{self.rows}", "device", device, "row0", row0)

    def _hash(self, epoch):
        # FAKE_CORRUPT_RANK: this rank's shard goes wrong from epoch 20 on
        # (a halo-exchange bug), which the summed hash must expose
        bad = 1 if self.corrupt and epoch >= 20 else 0
        return (self.board.block_sum(self.row0, self.rows, epoch) + bad) & M64

    def hash(self):
        log("hash", f"{self.w}x{self.rows}", self.epoch)
        return self._hash(self.epoch)

    def allreduce_u64(self, values):
        import torch
        import torch.distributed as dist
        v = np.asarray(values, dtype=np.uint64)
        lo = torch.tensor((v & np.uint64(0xFFFFFFFF)).astype(np.int64))
        hi = torch.tensor((v >> np.uint64(32)).astype(np.int64))
        dist.all_reduce(lo, group=_GROUP)
        dist.all_reduce(hi, group=_GROUP)
        log("allreduce", len(v))
        out = [((int(h) << 32) + int(l)) & M64 for l, h in zip(lo.tolist(), hi.tolist())]
        return np.array(out, dtype=np.uint64)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def close(self):
        log("close", f"{self.w}x{self.rows}")

    def set_tuning(self, band_rows=0, gens_per_pass=0, words_per_lane=0):
        pass

    def comm_init(self, uid, rank, world):
        log("comm_init", uid.hex()[:16], rank, world)
        if os.environ.get("FAKE_HANG_REJOIN") and world < int(os.environ.get("WORLD_SIZE", "1")):
            import time
            time.sleep(600)  # a ring rebuild that never completes (the drill's watchdog must end it)
        _join(rank, world)

    def comm_abort(self):
        log("comm_abort", f"{self.w}x{self.rows}")
        full = int(os.environ.get("WORLD_SIZE", "1"))
        if full > 1 and RANK == _lost_rank(full):
            import torch.distributed as dist
            dist.new_group([r for r in range(full) if r != RANK])  # collective: the survivors' next ring

    def seed(self, seed):
        self.epoch = 0
        log("seed", f"{self.w}x{self.rows}")

    def pass_plan(self, n, hashes=False):
        plan = [12] * (n // 12)
        return plan + [n % 12] if n % 12 else plan

    def load(self, packed):
        self.epoch = 0
        log("load", f"{self.w}x{self.rows}")

    def step(self, n, hashes=False):
        if self.ref_default is not None:
            e0 = self.epoch
            self.epoch += n
            return np.array(self.ref_default[e0:e0 + n], dtype=np.uint64) if hashes else None
        plan = self.pass_plan(n, hashes)
        self.gens += n
        self.launches += len(plan)
        self.ms += 1e-9 * self.w * self.rows * n / 100.0  # 100k GCUPS
        log("step", f"{self.w}x{self.rows}", n, "hashes" if hashes else "")
        e0 = self.epoch
        self.epoch += n
        if hashes:
            return np.array([self._hash(e0 + k + 1) for k in range(n)], dtype=np.uint64)
        return None

    def _my_rows(self, epoch):
        return FakeBoard.words(self.board.rows(np.arange(self.row0, self.row0 + self.rows), epoch))

    def snapshot(self, out=None):
        d = self._my_rows(self.epoch)
        if out is None:
            return d
        out[...] = d
        return out

    def checkpoint(self):
        if os.environ.get("FAKE_DRILL_RAISE") == str(RANK) and self.epoch == 20:
            raise OSError(28, "No space left on device")  # a checkpoint write that fails mid-drill
        from gameoflife.elastic import checkpoint_buffer
        blob, data = checkpoint_buffer(dict(width=self.w, height=self.h, row0=self.row0, epoch=self.epoch,
                                            topology=0, birth=8, survive=12), self.rows, 2)
        data[...] = self._my_rows(self.epoch)
        log("checkpoint", f"{self.w}x{self.rows}", self.row0, self.epoch)
        return blob

    def restore(self, blob):
        from gameoflife.elastic import parse_checkpoint
        h, data = parse_checkpoint(bytes(blob))
        if (h["width"], h["height"], h["row0"], h["rows"], h["wwords"]) != (self.w, self.h, self.row0, self.rows, 2):
            raise ValueError(f"checkpoint {h} does not fit the context {self.row0}+{self.rows}")
        if not np.array_equal(data, self._my_rows(h["epoch"])):
            raise ValueError(f"checkpoint rows {self.row0}+{self.rows} at epoch {h['epoch']} are not the board's")
        self.epoch = h["epoch"]
        log("restore", f"{self.w}x{self.rows}", self.row0, self.epoch)

    def replay(self, d, above, below):
        up = FakeBoard.words(self.board.rows(np.arange(self.row0 - d, self.row0), self.epoch))
        dn = FakeBoard.words(self.board.rows(np.arange(self.row0 + self.rows, self.row0 + self.rows + d), self.epoch))
        if not (np.array_equal(above, up) and np.array_equal(below, dn)):
            raise ValueError(f"light cone of rows {self.row0}+{self.rows} at epoch {self.epoch} is wrong")
        log("replay", f"{self.w}x{self.rows}", self.row0, self.epoch, d)
        return self.step(d, hashes=True)

    def sync(self):
        pass

    def profile(self, on):
        pass

    def profile_reset(self):
        self.gens = self.launches = 0
        self.ms = 0.0

    def profile_read(self):
        return self.ms, self.launches, self.gens

    def profile_clock(self):
        return 2.0 if self.launches else 0.0

    def profile_stats(self):
        sharded = not self.whole
        return {"kernel_ms": self.ms, "launches": self.launches, "generations": self.gens,
                "exchange_ms": 0.05 * self.launches if sharded else 0.0,
                "exchanges": self.launches if sharded else 0,
                "boundary_ms": 0.01 * self.launches if sharded else 0.0,
                "boundary_launches": self.launches if sharded else 0,
                "halo_bytes_sent": 2 * 12 * self.w // 8 * self.launches if sharded else 0,
                "halo_bytes_received": 2 * 12 * self.w // 8 * self.launches if sharded else 0,
                "clock_ghz": 2.0,
                "exchange_exposed_ms": 0.002 * self.launches if sharded else 0.0,
                "pass_tail_ms": 0.004 * self.launches if sharded else 0.0}

    def occupancy(self, g):
        return (12 if g > 8 else 16), 124


# The gloo group standing in for the current RCCL ring: the job's world at
# first; a later ring (the fault drill's survivors) gets a subgroup of the
# ranks still in it.  Group creation is collective over the whole job, so
# every rank -- the lost one included -- creates it: the lost rank does so
# when it drops its context (comm_abort is the last call it makes).
_GROUP = None


def _join(rank, world):
    global _GROUP
    import torch.distributed as dist
    full = int(os.environ.get("WORLD_SIZE", "1"))
    if world == full or world == 1 and full == 1:
        _GROUP = None  # the default group
        return
    lost = _lost_rank(full)
    _GROUP = dist.new_group([r for r in range(full) if r != lost])


def _lost_rank(full):
    return max(0, min(3, full - 1))


def install():
    native = types.ModuleType("gameoflife._native")
    native.GOL_UNIQUE_ID_BYTES = 128
    native.unique_id = lambda: bytes(range(128))

    def shard_rows(height, rank, n):
        base, extra = divmod(height, n)
        return rank * base + min(rank, extra), base + (1 if rank < extra else 0)

    native.shard_rows = shard_rows
    native.runtime_info = lambda: {"hip_runtime_version": 70226015, "hip_runtime": "7.2.26015",
                                   "hip_driver_version": 70226015, "rccl_version": 22707, "rccl": "2.27.7",
                                   "hip_library": "/opt/rocm/lib/libamdhip64.so.7",
                                   "rccl_library": "/opt/rocm/lib/librccl.so.1", "gol_library": "fake",
                                   "torch_loaded": "torch" in sys.modules}
    native.absorbed = lambda: (0, "")
    native.device_layout = lambda width, topology=0: 2 if (width // 32) % 2 == 0 else 1
    engine = types.ModuleType("gameoflife.engine")
    engine.GolEngine = FakeEngine
    pkg = types.ModuleType("gameoflife")
    pkg._native, pkg.engine = native, engine
    # the pure-Python modules (elastic: the fault drill's checkpoint files and
    # light cones; shard) load from the real package, around the stand-ins
    pkg.__path__ = [os.path.join(ROOT, "akka-game-of-life_amd", "gameoflife")]
    sys.modules.update({"gameoflife": pkg, "gameoflife._native": native, "gameoflife.engine": engine})
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:  # the stand-in for the engine's RCCL all-reduce
        import torch.distributed as dist
        saved = os.dup(1)  # gloo's connection banner goes to fd 1: keep stdout for the JSON line
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", rank=RANK, world_size=world)
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)


if __name__ == "__main__":
    if os.environ.get("FAKE_NO_ROOM"):  # no directory has room for the fault drill's checkpoint files
        import shutil
        shutil.disk_usage = lambda d: types.SimpleNamespace(total=1 << 30, used=1 << 30, free=0)
    install()
    sys.path.insert(0, ROOT)
    import bench
    sys.argv = ["bench.py"] + sys.argv[1:]
    try:
        bench.main()
    finally:
        if "torch.distributed" in sys.modules:  # the stand-in all-reduce's group: tear it down before exit
            import torch.distributed as dist
            if dist.is_initialized():
                dist.destroy_process_group()
