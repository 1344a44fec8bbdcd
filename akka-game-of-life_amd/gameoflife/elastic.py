"""Cross-process fault path: backends as processes, one lost mid-run.

Reference behaviour (BASELINE.json config 5): a
backend JVM dies (Ctrl-C in ``README.md:12``), the cluster downs it after 1 s
(``application.conf:23``), DeathWatch reports each of its cells
``Terminated`` and ``BoardCreator.onCellTermination`` re-deploys them on a
surviving backend, where they replay from the epoch-0 state and their
neighbours' never-pruned histories (``BoardCreator.scala:120-154``,
``CellActor.scala:34,71-74,86``).

Here a backend is one process per GPU that owns a row block (``GpuShard``:
a libgol context, halo rows over RCCL).  Every ``ckpt_every`` generations
each backend writes its shard checkpoint (``gol_checkpoint``) to a shared
directory.  The ``Supervisor`` plays the frontend: it starts the backends,
watches their progress, can inject a crash into one of them (the backend
SIGKILLs itself once it has advanced to the given generation -- the
analogue of the reference's injected ``DoCrashMsg``, ``BoardCreator.scala:
97-102``, but the whole process is gone), notices the loss, stops the rest
(their RCCL ring is broken), and re-deploys the whole board on the
survivors: the new row
blocks of the smaller decomposition are assembled from the last complete
checkpoint written by the old one, and the lost generations are replayed.
Generations are a pure function of that checkpoint, so the per-generation
state hashes equal those of an uninterrupted run.

Each backend is ``python -m gameoflife.elastic worker ...``; the shard
implementation is pluggable (``--shard module:Class``) so the CPU tests can
run the same supervisor and worker loop with a test double.

    python -m gameoflife.elastic demo --width 262144 --height 262144 \\
        --gens 50 --every 10 --world 8 --kill 3@25 --workdir /tmp/gol_fault
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import signal
import struct
import subprocess
import sys
import time

import numpy as np

from .shard import shard_rows_py

# CkptHeader of gol_capi.cpp: magic[8], width, height, row0, rows, wwords,
# epoch, topology, birth, survive, pad
_HDR = struct.Struct("<8s5qQiIIi")
_MAGIC = b"GOLCKPT1"


# ----------------------------------------------------------- checkpoints

def parse_checkpoint(blob: bytes) -> tuple[dict, np.ndarray]:
    """Header fields and packed rows (rows x wwords) of a gol_checkpoint blob."""
    magic, width, height, row0, rows, wwords, epoch, topology, birth, survive, _ = \
        _HDR.unpack_from(blob, 0)
    if magic != _MAGIC:
        raise ValueError("not a libgol checkpoint")
    h = dict(width=width, height=height, row0=row0, rows=rows, wwords=wwords, epoch=epoch,
             topology=topology, birth=birth, survive=survive)
    data = np.frombuffer(blob, dtype=np.uint32, count=rows * wwords, offset=_HDR.size)
    return h, data.reshape(rows, wwords)


def make_checkpoint(h: dict, packed: np.ndarray) -> bytes:
    """A gol_checkpoint blob for header fields `h` and rows `packed`."""
    rows, wwords = packed.shape
    hdr = _HDR.pack(_MAGIC, h["width"], h["height"], h["row0"], rows, wwords, h["epoch"],
                    h["topology"], h["birth"], h["survive"], 0)
    return hdr + np.ascontiguousarray(packed, dtype=np.uint32).tobytes()


def epoch_dir(ckpt_dir: str, epoch: int) -> str:
    return os.path.join(ckpt_dir, f"e{epoch:09d}")


def write_shard_checkpoint(ckpt_dir: str, blob: bytes) -> str:
    """Write one shard's checkpoint atomically (tmp + rename)."""
    h, _ = parse_checkpoint(blob)
    d = epoch_dir(ckpt_dir, h["epoch"])
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f"r{h['row0']:010d}_{h['rows']}.gol")
    tmp = path + f".tmp{os.getpid()}"
    with open(tmp, "wb") as f:
        f.write(blob)
    os.replace(tmp, path)
    return path


def _shard_files(ckpt_dir: str, epoch: int) -> list[tuple[int, int, str]]:
    d = epoch_dir(ckpt_dir, epoch)
    out = []
    for name in os.listdir(d) if os.path.isdir(d) else []:
        if name.startswith("r") and name.endswith(".gol"):
            row0, rows = name[1:-4].split("_")
            out.append((int(row0), int(rows), os.path.join(d, name)))
    return sorted(out)


def complete_epochs(ckpt_dir: str, height: int) -> list[int]:
    """Checkpoint epochs whose shard files tile rows [0, height) exactly."""
    out = []
    for name in sorted(os.listdir(ckpt_dir)) if os.path.isdir(ckpt_dir) else []:
        if not name.startswith("e"):
            continue
        epoch, nxt = int(name[1:]), 0
        for row0, rows, _ in _shard_files(ckpt_dir, epoch):
            if row0 != nxt:
                break
            nxt = row0 + rows
        if nxt == height:
            out.append(epoch)
    return out


def assemble_checkpoint(ckpt_dir: str, epoch: int, row0: int, rows: int) -> bytes:
    """Checkpoint blob for rows [row0, row0 + rows) at `epoch`, cut from the
    shard files of whatever decomposition wrote that epoch."""
    parts, header = [], None
    for f0, fn, path in _shard_files(ckpt_dir, epoch):
        lo, hi = max(row0, f0), min(row0 + rows, f0 + fn)
        if lo >= hi:
            continue
        with open(path, "rb") as f:
            h, data = parse_checkpoint(f.read())
        header = h
        parts.append((lo, data[lo - f0:hi - f0]))
    if header is None:
        raise FileNotFoundError(f"no checkpoint rows for [{row0}, {row0 + rows}) at epoch {epoch}")
    parts.sort(key=lambda p: p[0])
    packed = np.vstack([p[1] for p in parts])
    if packed.shape[0] != rows:
        raise ValueError(f"checkpoint at epoch {epoch} covers {packed.shape[0]} of {rows} rows")
    header = dict(header, row0=row0, rows=rows)
    return make_checkpoint(header, packed)


# ----------------------------------------------------------- shards

class GpuShard:
    """The product backend: one libgol context on one GPU; halo rows and the
    per-generation hash reduction over RCCL (rank 0 publishes the unique id
    in the attempt directory)."""

    def __init__(self, width, height, row0, rows, rank, world, attempt_dir, topology="torus",
                 rule="life", device=None):
        from . import _native as N
        from .engine import GolEngine
        ndev = N.device_count()
        self.world = world
        self.eng = GolEngine(width, height, topology=topology, rule=rule,
                             device=rank % ndev if device is None else device, row0=row0, rows=rows)
        if world > 1:
            uid_path = os.path.join(attempt_dir, "rccl_uid")
            if rank == 0:
                uid = N.unique_id()
                tmp = uid_path + ".tmp"
                with open(tmp, "wb") as f:
                    f.write(uid)
                os.replace(tmp, uid_path)
            else:
                deadline = time.time() + 120
                while not os.path.exists(uid_path):
                    if time.time() > deadline:
                        raise TimeoutError("no RCCL unique id from rank 0")
                    time.sleep(0.05)
                uid = open(uid_path, "rb").read()
            self.eng.comm_init(uid, rank, world)

    def seed(self, seed):
        self.eng.seed(seed)

    def restore(self, blob):
        self.eng.restore(blob)

    def checkpoint(self):
        return self.eng.checkpoint()

    def step(self, n):
        part = self.eng.step(n, hashes=True)
        return self.eng.allreduce_u64(part) if self.world > 1 else part

    def close(self):
        self.eng.close()


def _load_class(spec: str):
    mod, cls = spec.split(":")
    return getattr(importlib.import_module(mod), cls)


# ----------------------------------------------------------- backend process

def worker_main(a) -> int:
    row0, rows = shard_rows_py(a.height, a.rank, a.world)
    shard = _load_class(a.shard)(a.width, a.height, row0, rows, a.rank, a.world, a.attempt_dir,
                                 topology=a.topology, rule=a.rule)
    progress = os.path.join(a.attempt_dir, f"progress_r{a.rank}")
    hashes = open(os.path.join(a.attempt_dir, "hashes.txt"), "a") if a.rank == 0 else None

    def report(epoch):
        with open(progress + ".tmp", "w") as f:
            f.write(str(epoch))
        os.replace(progress + ".tmp", progress)

    if a.start == 0:
        shard.seed(a.seed)
        write_shard_checkpoint(a.ckpt_dir, shard.checkpoint())
    else:
        shard.restore(assemble_checkpoint(a.ckpt_dir, a.start, row0, rows))
    epoch = a.start
    report(epoch)
    while epoch < a.gens:
        n = min(a.chunk, a.every - epoch % a.every, a.gens - epoch)
        hs = shard.step(n)
        if hashes:
            for k, h in enumerate(hs):
                hashes.write(f"{epoch + k + 1} {int(h)}\n")
            hashes.flush()
        epoch += n
        if 0 <= a.crash_at <= epoch:  # injected crash: the process dies here
            os.kill(os.getpid(), signal.SIGKILL)
        if epoch % a.every == 0:
            write_shard_checkpoint(a.ckpt_dir, shard.checkpoint())
        report(epoch)
    shard.close()
    return 0


# ----------------------------------------------------------- supervisor

class Supervisor:
    """The frontend's role: deploy the board on `world` backends, optionally
    crash backend `kill = (rank, generation)` once it has advanced that far
    (before it writes a checkpoint there), and on
    any backend loss re-deploy on the survivors from the last complete
    checkpoint.  `hashes()` maps every generation to the global state hash
    (replayed generations overwrite the lost run's)."""

    def __init__(self, width, height, gens, world, workdir, ckpt_every=10, seed=0x5EED,
                 topology="torus", rule="life", shard="gameoflife.elastic:GpuShard", chunk=1,
                 kill=None, timeout=600.0, env=None):
        self.width, self.height, self.gens, self.world = width, height, gens, world
        self.workdir, self.every, self.seed = workdir, ckpt_every, seed
        self.topology, self.rule, self.shard, self.chunk = topology, rule, shard, chunk
        self.kill = kill  # (rank, epoch) or None
        self.timeout = timeout
        self.env = dict(os.environ if env is None else env)
        pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        self.env["PYTHONPATH"] = os.pathsep.join([pkg] + [p for p in self.env.get("PYTHONPATH", "").split(
            os.pathsep) if p])
        self.ckpt_dir = os.path.join(workdir, "ckpt")
        self.events: list[dict] = []
        self.attempts: list[str] = []

    def _launch(self, attempt, world, start, crash=None):
        d = os.path.join(self.workdir, f"attempt{attempt}")
        os.makedirs(d, exist_ok=True)
        self.attempts.append(d)
        procs = []
        for r in range(world):
            cmd = [sys.executable, "-m", "gameoflife.elastic", "worker",
                   "--width", str(self.width), "--height", str(self.height), "--gens", str(self.gens),
                   "--every", str(self.every), "--seed", str(self.seed), "--rank", str(r),
                   "--world", str(world), "--start", str(start), "--ckpt-dir", self.ckpt_dir,
                   "--attempt-dir", d, "--topology", self.topology, "--rule", self.rule,
                   "--shard", self.shard, "--chunk", str(self.chunk),
                   "--crash-at", str(crash[1] if crash and crash[0] == r else -1)]
            log = open(os.path.join(d, f"worker_r{r}.log"), "w")
            procs.append(subprocess.Popen(cmd, env=self.env, stdout=log, stderr=subprocess.STDOUT))
        self.events.append({"event": "deploy", "attempt": attempt, "world": world, "start": start})
        return d, procs

    @staticmethod
    def _progress(d, r):
        try:
            return int(open(os.path.join(d, f"progress_r{r}")).read() or -1)
        except (OSError, ValueError):
            return -1

    def run(self) -> dict:
        os.makedirs(self.workdir, exist_ok=True)
        deadline = time.time() + self.timeout
        world, start, attempt = self.world, 0, 0
        d, procs = self._launch(attempt, world, start, crash=self.kill)
        if self.kill:
            self.events.append({"event": "inject-crash", "rank": self.kill[0], "generation": self.kill[1]})
        try:
            while True:
                if time.time() > deadline:
                    raise TimeoutError("elastic run exceeded its time limit")
                codes = [p.poll() for p in procs]
                if all(c == 0 for c in codes):
                    break
                if any(c not in (None, 0) for c in codes):
                    lost = [r for r, c in enumerate(codes) if c not in (None, 0)]
                    progress = {r: self._progress(d, r) for r in range(len(procs))}
                    for p in procs:  # the ring is broken: stop the others too
                        if p.poll() is None:
                            p.send_signal(signal.SIGKILL)
                    for p in procs:
                        p.wait()
                    epochs = complete_epochs(self.ckpt_dir, self.height)
                    if not epochs:
                        raise RuntimeError("backend lost before the first checkpoint")
                    start = epochs[-1]
                    world = max(1, world - len(lost))
                    attempt += 1
                    self.events.append({"event": "lost", "ranks": lost, "progress": progress,
                                        "restart_epoch": start, "new_world": world})
                    d, procs = self._launch(attempt, world, start)
                    continue
                time.sleep(0.02)
        finally:
            for p in procs:
                if p.poll() is None:
                    p.send_signal(signal.SIGKILL)
                    p.wait()
        return self.hashes()

    def hashes(self) -> dict:
        out = {}
        for d in self.attempts:
            path = os.path.join(d, "hashes.txt")
            if os.path.exists(path):
                for line in open(path):
                    e, h = line.split()
                    out[int(e)] = int(h)
        return out


# ----------------------------------------------------------- CLI

def _parser():
    ap = argparse.ArgumentParser(prog="python -m gameoflife.elastic")
    sub = ap.add_subparsers(dest="cmd", required=True)
    w = sub.add_parser("worker", help="one backend process (started by the supervisor)")
    for name, typ in [("--width", int), ("--height", int), ("--gens", int), ("--every", int),
                      ("--seed", int), ("--rank", int), ("--world", int), ("--start", int),
                      ("--chunk", int), ("--crash-at", int)]:
        w.add_argument(name, type=typ, required=True)
    for name in ("--ckpt-dir", "--attempt-dir", "--topology", "--rule", "--shard"):
        w.add_argument(name, required=True)
    dm = sub.add_parser("demo", help="BASELINE.json config 5: kill one backend mid-run")
    dm.add_argument("--width", type=int, default=262144)
    dm.add_argument("--height", type=int, default=262144)
    dm.add_argument("--gens", type=int, default=50)
    dm.add_argument("--every", type=int, default=10)
    dm.add_argument("--world", type=int, default=8)
    dm.add_argument("--kill", default="3@25", help="crash rank@generation, or 'none'")
    dm.add_argument("--workdir", default="/tmp/gol_elastic")
    return ap


def main(argv=None) -> int:
    a = _parser().parse_args(argv)
    if a.cmd == "worker":
        return worker_main(a)
    kill = None if a.kill == "none" else tuple(int(x) for x in a.kill.split("@"))
    sup = Supervisor(a.width, a.height, a.gens, a.world, a.workdir, a.every, kill=kill, chunk=5)
    got = sup.run()
    ref = Supervisor(a.width, a.height, a.gens, a.world, a.workdir + "_ref", a.every, chunk=5).run()
    same = [got.get(e) == ref.get(e) for e in range(1, a.gens + 1)]
    print(json.dumps({"events": sup.events, "generations": a.gens, "hashes_equal": all(same)}))
    return 0 if all(same) else 1


if __name__ == "__main__":
    sys.exit(main())
