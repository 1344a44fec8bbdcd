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
    name = f"bench_{width}.json" if width == height else f"bench_{width}x{height}.json"
    with open(os.path.join(ROOT, "tests", "golden", name)) as f:
        return [int(x, 16) for x in json.load(f)["hashes"]]


class FakeEngine:
    """Records calls; its state hash is a share of the golden hash of its
    epoch: rank r > 0 holds a pseudo-random share, rank 0 the rest, so only
    the sum over all ranks (the all-reduce) equals the golden value."""

    def __init__(self, width, height, topology="torus", rule="life", device=0, row0=0, rows=0):
        self.w, self.h, self.rows = width, height, rows or height
        self.gens = self.launches = 0
        self.ms = 0.0
        self.epoch = 0
        self.whole = self.rows == height
        log("create", f"{width}x{self.rows}", "device", device, "row0", row0)

    def _share(self, epoch):
        world = int(os.environ.get("WORLD_SIZE", "1"))
        if self.whole or world == 1:
            g = golden(self.w, self.rows)
            return g[epoch] if epoch < len(g) else 0
        others = [(0x9E3779B97F4A7C15 * (epoch + 1) * (r + 7)) & M64 for r in range(1, world)]
        if RANK > 0:
            # FAKE_CORRUPT_RANK: this rank's shard goes wrong from epoch 20 on
            # (a halo-exchange bug), which the summed hash must expose
            bad = os.environ.get("FAKE_CORRUPT_RANK") == str(RANK) and epoch >= 20
            return (others[RANK - 1] + (1 if bad else 0)) & M64
        g = golden(self.w, self.h)
        return ((g[epoch] if epoch < len(g) else 0) - sum(others)) & M64

    def hash(self):
        log("hash", f"{self.w}x{self.rows}", self.epoch)
        return self._share(self.epoch)

    def allreduce_u64(self, values):
        import torch
        import torch.distributed as dist
        v = np.asarray(values, dtype=np.uint64)
        lo = torch.tensor((v & np.uint64(0xFFFFFFFF)).astype(np.int64))
        hi = torch.tensor((v >> np.uint64(32)).astype(np.int64))
        dist.all_reduce(lo)
        dist.all_reduce(hi)
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

    def seed(self, seed):
        self.epoch = 0
        log("seed", f"{self.w}x{self.rows}")

    def pass_plan(self, n, hashes=False):
        plan = [12] * (n // 12)
        return plan + [n % 12] if n % 12 else plan

    def step(self, n, hashes=False):
        plan = self.pass_plan(n, hashes)
        self.gens += n
        self.launches += len(plan)
        self.ms += 1e-9 * self.w * self.rows * n / 100.0  # 100k GCUPS
        log("step", f"{self.w}x{self.rows}", n, "hashes" if hashes else "")
        e0 = self.epoch
        self.epoch += n
        if hashes:
            return np.array([self._share(e0 + k + 1) for k in range(n)], dtype=np.uint64)
        return None

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
