"""Runs bench.py's main() with a stand-in for libgol (test infrastructure for
tests/test_bench_multirank.py, not a test module).

The N > 1 control flow of bench.py -- gloo process group, communicator-id
broadcast, barriers, max-over-ranks time, the per-rank 65536^2 run, the one
JSON line on rank 0 -- only runs for real on the driver's multi-GPU node.
This runner replaces the native engine by a recorder so that flow can run on
CPU ranks: every engine call is appended to $FAKE_LOG_DIR/rank<r>.log.

    RANK=.. WORLD_SIZE=.. MASTER_ADDR=127.0.0.1 MASTER_PORT=.. FAKE_LOG_DIR=.. \
        python tests/bench_fake_runner.py --gpus N --steps K --warmup W ...
"""
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RANK = int(os.environ.get("RANK", "0"))
LOG = os.path.join(os.environ["FAKE_LOG_DIR"], f"rank{RANK}.log")


def log(*parts):
    with open(LOG, "a") as f:
        f.write(" ".join(str(p) for p in parts) + "\n")


class FakeEngine:
    def __init__(self, width, height, topology="torus", rule="life", device=0, row0=0, rows=0):
        self.w, self.h, self.rows = width, height, rows or height
        self.gens = self.launches = 0
        self.ms = 0.0
        log("create", f"{width}x{self.rows}", "device", device, "row0", row0)

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
    engine = types.ModuleType("gameoflife.engine")
    engine.GolEngine = FakeEngine
    pkg = types.ModuleType("gameoflife")
    pkg._native, pkg.engine = native, engine
    sys.modules.update({"gameoflife": pkg, "gameoflife._native": native, "gameoflife.engine": engine})
    import torch
    torch.cuda.set_device = lambda d: log("set_device", d)
    torch.cuda.synchronize = lambda *a: None


if __name__ == "__main__":
    install()
    sys.path.insert(0, ROOT)
    import bench
    sys.argv = ["bench.py"] + sys.argv[1:]
    bench.main()
