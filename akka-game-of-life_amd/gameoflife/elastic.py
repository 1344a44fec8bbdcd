"""Cross-process fault path: backends as processes, lost ones re-spawned alone.

Reference behaviour (BASELINE.json config 5): a
backend JVM dies (Ctrl-C in ``README.md:12``) or a cell is crashed on purpose
(``crashIfIMay``, every ``errors.every`` after ``errors.delay`` up to
``max-crashes``, ``BoardCreator.scala:97-102,108``).  DeathWatch reports the
cell ``Terminated`` and ``BoardCreator.onCellTermination`` re-deploys only
that cell, on a surviving node (``BoardCreator.scala:120-154``); it replays
from its epoch-0 state using its neighbours' never-pruned histories
(``CellActor.scala:34,71-74,86``) while every other cell keeps its state and
simply waits for the answers it needs.

Here a backend is one process per GPU owning a row block (``GpuShard``: a
libgol context, halo rows over RCCL).  Every ``ckpt_every`` generations each
backend writes its shard checkpoint (``gol_checkpoint``) to a shared
directory.  The ``Supervisor`` plays the frontend: it starts the backends and
releases them chunk by chunk (a backend only enters the next ring exchange
when the supervisor says go, so when one dies the others are parked between
steps, never inside a collective).  When a backend is lost at epoch t:

* its row block is re-spawned on a surviving GPU -- the backend whose rows
  are adjacent to it absorbs it: it restores the lost block's checkpoint at
  epoch c <= t, takes the t - c rows above and below it at epoch c from the
  neighbours' checkpoint files (the light cone), and replays the block alone
  to epoch t (``gol_replay``), then owns both blocks as one context;
* nobody else rolls back: the survivors stay at epoch t;
* the ring is rebuilt around the merged backend (``gol_comm_abort`` +
  ``gol_comm_init`` with a new unique id) and the run continues.

The replayed block's per-generation partial hashes are checked against the
global hashes recorded before the loss minus the survivors' partials.  If the
last backend dies, a fresh one restores the whole board from the checkpoint
files and replays it to epoch t the same way.

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

# CkptHeader of gol_ctx.h: magic[8], width, height, row0, rows, wwords,
# epoch, topology, birth, survive, pad
_HDR = struct.Struct("<8s5qQiIIi")
_MAGIC = b"GOLCKPT1"


# ----------------------------------------------------------- checkpoints

def _header(blob) -> dict:
    if len(blob) < _HDR.size:
        raise ValueError("not a libgol checkpoint")
    magic, width, height, row0, rows, wwords, epoch, topology, birth, survive, _ = \
        _HDR.unpack_from(blob, 0)
    if magic != _MAGIC:
        raise ValueError("not a libgol checkpoint")
    return dict(width=width, height=height, row0=row0, rows=rows, wwords=wwords, epoch=epoch,
                topology=topology, birth=birth, survive=survive)


def parse_checkpoint(blob: bytes) -> tuple[dict, np.ndarray]:
    """Header fields and packed rows (rows x wwords) of a gol_checkpoint blob."""
    h = _header(blob)
    data = np.frombuffer(blob, dtype=np.uint32, count=h["rows"] * h["wwords"], offset=_HDR.size)
    return h, data.reshape(h["rows"], h["wwords"])


def read_checkpoint_header(path: str) -> dict:
    """Header fields of a checkpoint file, without reading its rows."""
    with open(path, "rb") as f:
        return _header(f.read(_HDR.size))


def make_checkpoint(h: dict, packed: np.ndarray) -> bytes:
    """A gol_checkpoint blob for header fields `h` and rows `packed`."""
    rows, wwords = packed.shape
    hdr = _HDR.pack(_MAGIC, h["width"], h["height"], h["row0"], rows, wwords, h["epoch"],
                    h["topology"], h["birth"], h["survive"], 0)
    return hdr + np.ascontiguousarray(packed, dtype=np.uint32).tobytes()


def checkpoint_buffer(h: dict, rows: int, wwords: int) -> tuple[np.ndarray, np.ndarray]:
    """An empty gol_checkpoint blob for header fields `h` (row0, epoch, ...)
    and `rows` rows: (the blob as uint8, its rows as a (rows, wwords) uint32
    view to fill in place -- snapshot(out=...) slices -- with no extra copy)."""
    blob = np.empty(_HDR.size + rows * wwords * 4, dtype=np.uint8)
    _HDR.pack_into(blob, 0, _MAGIC, h["width"], h["height"], h["row0"], rows, wwords, h["epoch"], h["topology"],
                   h["birth"], h["survive"], 0)
    return blob, blob[_HDR.size:].view(np.uint32).reshape(rows, wwords)


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


def _covers(files: list[tuple[int, int, str]], lo: int, hi: int) -> bool:
    """Do the files' row blocks cover [lo, hi)?  Blocks may overlap: every
    file of one epoch holds that epoch's true rows (the board at an epoch is a
    pure function of the initial board), whichever decomposition wrote it."""
    nxt = lo
    for row0, rows, _ in sorted(files):
        if row0 > nxt:
            break
        nxt = max(nxt, row0 + rows)
    return nxt >= hi


def complete_epochs(ckpt_dir: str, height: int) -> list[int]:
    """Checkpoint epochs whose shard files cover rows [0, height)."""
    out = []
    for name in sorted(os.listdir(ckpt_dir)) if os.path.isdir(ckpt_dir) else []:
        if name.startswith("e") and _covers(_shard_files(ckpt_dir, int(name[1:])), 0, height):
            out.append(int(name[1:]))
    return out


def covering_epochs(ckpt_dir: str, lo: int, hi: int) -> list[int]:
    """Checkpoint epochs whose files cover rows [lo, hi)."""
    out = []
    for name in sorted(os.listdir(ckpt_dir)) if os.path.isdir(ckpt_dir) else []:
        if name.startswith("e") and _covers(_shard_files(ckpt_dir, int(name[1:])), lo, hi):
            out.append(int(name[1:]))
    return out


def light_cone_ranges(lo: int, hi: int, depth: int, height: int, torus: bool) -> list[tuple[int, int]]:
    """Row intervals of [0, height) that block [lo, hi) and its `depth`-row
    light cone on each side occupy (mod the height on a torus, clipped at a
    clipped board's edges)."""
    a, b = lo - depth, hi + depth
    if not torus:
        return [(max(a, 0), min(b, height))]
    n = b - a
    if n >= height:
        return [(0, height)]
    a %= height
    return [(a, a + n)] if a + n <= height else [(a, height), (0, a + n - height)]


def recovery_epoch(ckpt_dir: str, lo: int, hi: int, epoch: int, height: int, torus: bool) -> int:
    """The latest checkpoint epoch c <= `epoch` from which block [lo, hi) can
    be replayed to `epoch`: the files of c must hold the block AND its light
    cone, the epoch - c rows on each side.  The block's own file alone is not
    enough -- a backend killed at a checkpoint epoch dies before writing its
    file, so a neighbour lost later may find its own rows at an epoch whose
    light cone is incomplete."""
    for c in sorted((e for e in covering_epochs(ckpt_dir, lo, hi) if e <= epoch), reverse=True):
        files = _shard_files(ckpt_dir, c)
        if all(_covers(files, a, b) for a, b in light_cone_ranges(lo, hi, epoch - c, height, torus)):
            return c
    raise FileNotFoundError(f"no checkpoint epoch <= {epoch} holds rows [{lo}, {hi}) and their light cone")


def blob_rows(blobs, indices) -> np.ndarray:
    """Rows `indices` (global row numbers) cut from checkpoint blobs of one
    epoch (any decomposition; blocks may overlap)."""
    idx = np.asarray(list(indices), dtype=np.int64)
    out, done = None, np.zeros(idx.size, dtype=bool)
    for blob in blobs:
        h, data = parse_checkpoint(blob)
        f0, fn = h["row0"], h["rows"]
        if out is None:
            out = np.zeros((idx.size, data.shape[1]), dtype=np.uint32)
        sel = (~done) & (idx >= f0) & (idx < f0 + fn)
        out[sel] = data[idx[sel] - f0]
        done |= sel
    if out is None or not done.all():
        raise ValueError(f"checkpoints do not hold rows {idx[~done][:4].tolist()}...")
    return out


def checkpoint_rows(ckpt_dir: str, epoch: int, indices) -> np.ndarray:
    """Rows `indices` (global row numbers in [0, height)) of the board at
    `epoch`, cut from whatever shard files hold them.  Only the rows asked
    for are read (a light cone is a few rows of a file that may hold a GiB):
    each file's header, then one read per run of consecutive rows."""
    idx = np.asarray(list(indices), dtype=np.int64)
    out, done = None, np.zeros(idx.size, dtype=bool)
    for f0, fn, path in _shard_files(ckpt_dir, epoch):
        sel = np.nonzero((~done) & (idx >= f0) & (idx < f0 + fn))[0]
        if sel.size == 0:
            continue
        with open(path, "rb") as f:
            h = _header(f.read(_HDR.size))
            if h["row0"] != f0 or h["rows"] != fn:
                raise ValueError(f"{path}: not the checkpoint its name says")
            wwords = h["wwords"]
            if out is None:
                out = np.zeros((idx.size, wwords), dtype=np.uint32)
            order = sel[np.argsort(idx[sel], kind="stable")]
            k = 0
            while k < order.size:  # runs of consecutive rows: one read each
                j = k
                while j + 1 < order.size and idx[order[j + 1]] == idx[order[j]] + 1:
                    j += 1
                r_lo = int(idx[order[k]])
                f.seek(_HDR.size + (r_lo - f0) * wwords * 4)
                data = np.frombuffer(f.read((j - k + 1) * wwords * 4), dtype=np.uint32).reshape(-1, wwords)
                out[order[k:j + 1]] = data
                k = j + 1
        done[sel] = True
    if out is None or not done.all():
        raise FileNotFoundError(f"epoch {epoch}: checkpoints do not hold rows {idx[~done][:4].tolist()}...")
    return out


def assemble_checkpoint(ckpt_dir: str, epoch: int, row0: int, rows: int) -> bytes:
    """Checkpoint blob for rows [row0, row0 + rows) at `epoch`, cut from the
    shard files of whatever decomposition wrote that epoch."""
    files = _shard_files(ckpt_dir, epoch)
    if not files:
        raise FileNotFoundError(f"no checkpoint at epoch {epoch}")
    header = read_checkpoint_header(files[0][2])
    packed = checkpoint_rows(ckpt_dir, epoch, range(row0, row0 + rows))
    return make_checkpoint(dict(header, row0=row0, rows=rows, epoch=epoch), packed)


def light_cone_from(get_rows, row0: int, rows: int, depth: int, height: int, torus: bool,
                    wwords: int) -> tuple[np.ndarray, np.ndarray]:
    """The `depth` rows above row0 and below row0 + rows (mod the height on a
    torus; dead rows beyond a clipped board's edge), read with
    get_rows(global row indices): with the block's own rows they fix the block
    for `depth` generations (gol_replay)."""
    res = []
    for idx in ([row0 - depth + k for k in range(depth)], [row0 + rows + k for k in range(depth)]):
        if torus:
            res.append(get_rows([i % height for i in idx]) if idx else np.zeros((0, wwords), np.uint32))
            continue
        a = np.zeros((len(idx), wwords), dtype=np.uint32)
        inside = [k for k, i in enumerate(idx) if 0 <= i < height]
        if inside:
            a[inside] = get_rows([idx[k] for k in inside])
        res.append(a)
    return res[0], res[1]


def light_cone(ckpt_dir: str, epoch: int, row0: int, rows: int, depth: int, height: int,
               torus: bool) -> tuple[np.ndarray, np.ndarray]:
    """light_cone_from the checkpoint files of `epoch`."""
    files = _shard_files(ckpt_dir, epoch)
    if not files:
        raise FileNotFoundError(f"no checkpoint at epoch {epoch}")
    wwords = read_checkpoint_header(files[0][2])["wwords"]
    return light_cone_from(lambda idx: checkpoint_rows(ckpt_dir, epoch, idx), row0, rows, depth, height, torus,
                           wwords)


# ----------------------------------------------------------- shards

class GpuShard:
    """The product backend: one libgol context on one GPU; halo rows and the
    per-generation hash reduction over RCCL (the ring's rank 0 publishes the
    unique id in the ring directory)."""

    def __init__(self, width, height, row0, rows, topology="torus", rule="life", device=0):
        from .engine import GolEngine
        self.width, self.height, self.row0, self.rows = width, height, row0, rows
        self.topology, self.rule, self.device = topology, rule, device
        self.world = 1
        self.eng = GolEngine(width, height, topology=topology, rule=rule, device=device, row0=row0, rows=rows)

    def join(self, ring_dir, rank, world):
        """Join the ring `ring_dir` as rank/world (a 1-rank ring needs none)."""
        from . import _native as N
        self.world = world
        if world == 1:
            return
        uid = _ring_uid(ring_dir, rank, N.unique_id)
        self.eng.comm_init(uid, rank, world)

    def leave(self):
        self.eng.comm_abort()
        self.world = 1

    def seed(self, seed):
        self.eng.seed(seed)

    def restore(self, blob):
        self.eng.restore(blob)

    def checkpoint(self):
        return self.eng.checkpoint()

    def step(self, n):
        """-> (global per-generation hashes, this shard's partials)."""
        part = self.eng.step(n, hashes=True)
        return (self.eng.allreduce_u64(part) if self.world > 1 else part), part

    def close(self):
        self.eng.close()

    @staticmethod
    def replay_block(width, height, blob, above, below, depth, topology="torus", rule="life", device=0):
        """Light-cone replay of a lost block (gol_replay) on `device`:
        -> (the block's rows `depth` generations later, its partial hashes)."""
        from .engine import GolEngine
        h, _ = parse_checkpoint(blob)
        with GolEngine(width, height, topology=topology, rule=rule, device=device, row0=h["row0"],
                       rows=h["rows"]) as e:
            e.restore(blob)
            hs = e.replay(depth, above, below) if depth else np.zeros(0, dtype=np.uint64)
            return e.snapshot(), hs


def _ring_uid(ring_dir, rank, make_uid) -> bytes:
    """Rank 0 publishes the ring's unique id; the others wait for it."""
    path = os.path.join(ring_dir, "rccl_uid")
    if rank == 0:
        uid = make_uid()
        tmp = path + ".tmp"
        with open(tmp, "wb") as f:
            f.write(uid)
        os.replace(tmp, path)
        return uid
    deadline = time.time() + 120
    while not os.path.exists(path):
        if time.time() > deadline:
            raise TimeoutError("no ring unique id from rank 0")
        time.sleep(0.02)
    return open(path, "rb").read()


def _load_class(spec: str):
    mod, cls = spec.split(":")
    return getattr(importlib.import_module(mod), cls)


def _write_json(path, obj):
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(obj, f)
    os.replace(tmp, path)


def _read_json(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


# ----------------------------------------------------------- backend process

def worker_main(a) -> int:
    """One backend: runs the supervisor's commands (cmd/w<id>.<seq>, JSON)
    and reports after each one (status/w<id>)."""
    cls = _load_class(a.shard)
    torus = a.topology == "torus"
    row0, rows = a.row0, a.rows
    shard = cls(a.width, a.height, row0, rows, topology=a.topology, rule=a.rule, device=a.device)
    hashes = open(os.path.join(a.workdir, "hashes.txt"), "a")
    partials = open(os.path.join(a.workdir, f"partials_w{a.wid}.txt"), "a")
    status = os.path.join(a.workdir, "status", f"w{a.wid}")
    rank, world = a.rank, a.world
    extra = {}

    def report(seq, epoch):
        _write_json(status, dict(seq=seq, epoch=epoch, row0=row0, rows=rows, pid=os.getpid(), **extra))

    if a.resume < 0:
        shard.seed(a.seed)
        epoch = 0
        write_shard_checkpoint(a.ckpt_dir, shard.checkpoint())
    else:  # a re-spawned board: restore epoch c, replay to the target alone
        blob = assemble_checkpoint(a.ckpt_dir, a.resume, row0, rows)
        d = a.target - a.resume
        up, dn = light_cone(a.ckpt_dir, a.resume, row0, rows, d, a.height, torus)
        cur, hs = cls.replay_block(a.width, a.height, blob, up, dn, d, topology=a.topology, rule=a.rule,
                                   device=a.device)
        h, _ = parse_checkpoint(blob)
        shard.restore(make_checkpoint(dict(h, epoch=a.target), cur))
        epoch = a.target
        extra["replayed"] = {"from": a.resume, "to": a.target, "partials": [str(int(x)) for x in hs]}
        write_shard_checkpoint(a.ckpt_dir, shard.checkpoint())  # the next loss replays from here
    shard.join(a.ring_dir, rank, world)
    report(0, epoch)
    seq = 0
    while True:
        seq += 1
        path = os.path.join(a.workdir, "cmd", f"w{a.wid}.{seq}")
        while not os.path.exists(path):
            time.sleep(0.005)
        cmd = _read_json(path)
        while cmd is None:
            time.sleep(0.005)
            cmd = _read_json(path)
        op = cmd["op"]
        if op == "stop":
            shard.close()
            report(seq, epoch)
            return 0
        if op == "go":
            n = cmd["n"]
            glob, part = shard.step(n)
            if rank == 0:
                hashes.write("".join(f"{epoch + k + 1} {int(x)}\n" for k, x in enumerate(glob)))
                hashes.flush()
            partials.write("".join(f"{epoch + k + 1} {row0} {rows} {int(x)}\n" for k, x in enumerate(part)))
            partials.flush()
            epoch += n
            if cmd.get("crash"):  # injected crash (DoCrashMsg): the process dies here
                os.kill(os.getpid(), signal.SIGKILL)
            if epoch % a.every == 0:
                write_shard_checkpoint(a.ckpt_dir, shard.checkpoint())
        elif op == "absorb":
            # re-spawn the lost block next to this one: replay it alone from
            # its checkpoint with the light cone, then own both blocks
            lo, n_lost, c = cmd["row0"], cmd["rows"], cmd["ckpt_epoch"]
            d = epoch - c
            blob = assemble_checkpoint(a.ckpt_dir, c, lo, n_lost)
            up, dn = light_cone(a.ckpt_dir, c, lo, n_lost, d, a.height, torus)
            lost_rows, hs = cls.replay_block(a.width, a.height, blob, up, dn, d, topology=a.topology,
                                             rule=a.rule, device=a.device)
            mine_h, mine = parse_checkpoint(shard.checkpoint())
            shard.leave()
            shard.close()
            if lo + n_lost == row0:
                merged, row0 = np.vstack([lost_rows, mine]), lo
            elif row0 + rows == lo:
                merged = np.vstack([mine, lost_rows])
            else:
                raise ValueError(f"block [{lo}, {lo + n_lost}) is not adjacent to [{row0}, {row0 + rows})")
            rows += n_lost
            shard = cls(a.width, a.height, row0, rows, topology=a.topology, rule=a.rule, device=a.device)
            shard.restore(make_checkpoint(dict(mine_h, row0=row0, rows=rows, epoch=epoch), merged))
            extra["replayed"] = {"from": c, "to": epoch, "row0": lo, "rows": n_lost,
                                 "partials": [str(int(x)) for x in hs]}
            # the merged block's rows at this epoch, so a later loss next to
            # it finds a complete light cone without going back past it
            write_shard_checkpoint(a.ckpt_dir, shard.checkpoint())
            world = 1
        elif op == "rejoin":
            shard.leave()
            rank, world = cmd["rank"], cmd["world"]
            shard.join(cmd["ring"], rank, world)
        report(seq, epoch)


# ----------------------------------------------------------- supervisor

class _Worker:
    def __init__(self, wid, proc, row0, rows, rank, device):
        self.wid, self.proc, self.row0, self.rows, self.rank, self.device = wid, proc, row0, rows, rank, device
        self.seq = 0


class Supervisor:
    """The frontend's role: deploy the board on `world` backends, release them
    chunk by chunk, inject crashes, and re-spawn each lost block next to a
    survivor (lost-shard-only light-cone recovery, module docstring).

    crashes: [(generation, pick)] -- after `generation`, live backend number
    pick % live (in row order) dies (board.crash_schedule turns the
    reference's errors.delay / errors.every / max-crashes into this);
    kill = (rank, generation) is the one-crash shorthand.  `hashes()` maps
    every generation to the global state hash."""

    def __init__(self, width, height, gens, world, workdir, ckpt_every=10, seed=0x5EED,
                 topology="torus", rule="life", shard="gameoflife.elastic:GpuShard", chunk=1,
                 kill=None, crashes=None, timeout=600.0, env=None, devices=None):
        self.width, self.height, self.gens, self.world = width, height, gens, world
        self.workdir, self.every, self.seed = workdir, ckpt_every, seed
        self.topology, self.rule, self.shard, self.chunk = topology, rule, shard, chunk
        self.crashes = sorted(crashes or ([] if kill is None else [(kill[1], kill[0])]))
        self.timeout = timeout
        self.devices = list(devices) if devices is not None else None
        self.env = dict(os.environ if env is None else env)
        pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        self.env["PYTHONPATH"] = os.pathsep.join([pkg] + [p for p in self.env.get("PYTHONPATH", "").split(
            os.pathsep) if p])
        self.ckpt_dir = os.path.join(workdir, "ckpt")
        self.events: list[dict] = []
        self.workers: list[_Worker] = []
        self.next_wid = 0
        self.ring = 0
        self.deadline = 0.0

    # -- plumbing -----------------------------------------------------------
    def _device_count(self):
        if self.devices is None:
            try:
                from . import _native as N
                self.devices = list(range(max(1, N.device_count())))
            except Exception:
                self.devices = [0]
        return self.devices

    def _ring_dir(self):
        d = os.path.join(self.workdir, f"ring{self.ring}")
        os.makedirs(d, exist_ok=True)
        return d

    def _spawn(self, row0, rows, rank, world, device, resume=-1, target=-1):
        wid = self.next_wid
        self.next_wid += 1
        cmd = [sys.executable, "-m", "gameoflife.elastic", "worker",
               "--wid", str(wid), "--width", str(self.width), "--height", str(self.height),
               "--every", str(self.every), "--seed", str(self.seed), "--row0", str(row0), "--rows", str(rows),
               "--rank", str(rank), "--world", str(world), "--device", str(device),
               "--resume", str(resume), "--target", str(target), "--ring-dir", self._ring_dir(),
               "--workdir", self.workdir, "--ckpt-dir", self.ckpt_dir, "--topology", self.topology,
               "--rule", self.rule, "--shard", self.shard]
        log = open(os.path.join(self.workdir, "logs", f"worker_w{wid}.log"), "w")
        proc = subprocess.Popen(cmd, env=self.env, stdout=log, stderr=subprocess.STDOUT)
        w = _Worker(wid, proc, row0, rows, rank, device)
        self.workers.append(w)
        return w

    def _send(self, w, cmd):
        w.seq += 1
        _write_json(os.path.join(self.workdir, "cmd", f"w{w.wid}.{w.seq}"), cmd)

    def _wait(self, ws):
        """Wait until every worker in `ws` has reported its last command, or
        one of them died.  -> (statuses by wid, dead workers)."""
        while True:
            if time.time() > self.deadline:
                raise TimeoutError("elastic run exceeded its time limit")
            dead = [w for w in ws if w.proc.poll() not in (None, 0)]
            st = {w.wid: _read_json(os.path.join(self.workdir, "status", f"w{w.wid}")) for w in ws}
            done = all(st[w.wid] is not None and st[w.wid]["seq"] >= w.seq for w in ws if w not in dead)
            if done:
                return st, dead
            time.sleep(0.01)

    def _rering(self):
        """Renumber the live backends in row order and rebuild the ring."""
        self.workers.sort(key=lambda w: w.row0)
        self.ring += 1
        ring = self._ring_dir()
        for r, w in enumerate(self.workers):
            w.rank = r
            self._send(w, {"op": "rejoin", "ring": ring, "rank": r, "world": len(self.workers)})
        st, dead = self._wait(self.workers)
        if dead:
            raise RuntimeError("a backend died while the ring was rebuilt")
        return st

    # -- recovery -----------------------------------------------------------
    def _recover(self, lost: list[_Worker], epoch: int):
        for w in lost:
            self.workers.remove(w)
        for w in sorted(lost, key=lambda w: w.row0):
            c = recovery_epoch(self.ckpt_dir, w.row0, w.row0 + w.rows, epoch, self.height, self.topology == "torus")
            ev = {"event": "lost", "worker": w.wid, "rows": [w.row0, w.row0 + w.rows], "epoch": epoch,
                  "checkpoint_epoch": c, "replayed_generations": epoch - c}
            above = [s for s in self.workers if s.row0 + s.rows == w.row0]
            below = [s for s in self.workers if s.row0 == w.row0 + w.rows]
            host = (above or below or [None])[0]
            if host is None:  # the last backend: a fresh one for the whole board
                devs = self._device_count()
                nw = self._spawn(0, self.height, 0, 1, devs[(w.device + 1) % len(devs)], resume=c, target=epoch)
                st, dead = self._wait([nw])
                if dead:
                    raise RuntimeError("the re-spawned backend died")
                ev.update(respawned_as=nw.wid, device=nw.device, new_world=1)
                self._check_replay(st[nw.wid]["replayed"], epoch)
            else:
                self._send(host, {"op": "absorb", "row0": w.row0, "rows": w.rows, "ckpt_epoch": c})
                st, dead = self._wait([host])
                if dead:
                    raise RuntimeError("the absorbing backend died")
                host.row0, host.rows = st[host.wid]["row0"], st[host.wid]["rows"]
                ev.update(absorbed_by=host.wid, device=host.device, new_world=len(self.workers))
                self._check_replay(st[host.wid]["replayed"], epoch)
            self.events.append(ev)
        self._rering()

    def _check_replay(self, rep, epoch):
        """The replayed block's partial hashes must complete the global hashes
        recorded before the loss (sum of the other blocks' partials + it)."""
        part = self._partials()
        glob = self.hashes()
        lo, rows = rep.get("row0", 0), rep.get("rows", self.height)
        for k, p in enumerate(rep["partials"]):
            g = rep["from"] + k + 1
            if g not in glob:
                continue
            others = sum(v for (r0, n), v in part.get(g, {}).items() if r0 + n <= lo or r0 >= lo + rows)
            if (others + int(p)) % (1 << 64) != glob[g]:
                raise AssertionError(f"replayed partial of generation {g} does not complete the global hash")

    def _partials(self) -> dict:
        out: dict = {}
        logs = os.path.join(self.workdir)
        for name in os.listdir(logs):
            if name.startswith("partials_w"):
                for line in open(os.path.join(logs, name)):
                    g, r0, n, h = (int(x) for x in line.split())
                    out.setdefault(g, {})[(r0, n)] = h
        return out

    # -- main loop ----------------------------------------------------------
    def run(self) -> dict:
        for sub in ("cmd", "status", "logs"):
            os.makedirs(os.path.join(self.workdir, sub), exist_ok=True)
        self.deadline = time.time() + self.timeout
        devs = self._device_count()
        for r in range(self.world):
            row0, rows = shard_rows_py(self.height, r, self.world)
            self._spawn(row0, rows, r, self.world, devs[r % len(devs)])
        self.events.append({"event": "deploy", "world": self.world})
        pending = list(self.crashes)
        try:
            st, dead = self._wait(self.workers)
            if dead:
                raise RuntimeError("a backend died during deployment")
            epoch = 0
            while epoch < self.gens:
                while pending and pending[0][0] <= epoch:
                    pending.pop(0)
                n = min(self.chunk, self.every - epoch % self.every, self.gens - epoch)
                victim = None
                if pending and epoch + n >= pending[0][0]:
                    n = pending[0][0] - epoch
                    victim = sorted(self.workers, key=lambda w: w.row0)[pending[0][1] % len(self.workers)]
                    self.events.append({"event": "inject-crash", "worker": victim.wid, "generation": epoch + n})
                for w in self.workers:
                    self._send(w, {"op": "go", "n": n, "crash": w is victim})
                st, dead = self._wait(self.workers)
                for w in dead:
                    w.proc.wait()
                epoch += n
                if dead:
                    self._recover(dead, epoch)
            for w in self.workers:
                self._send(w, {"op": "stop"})
            self._wait(self.workers)
            for w in self.workers:
                if w.proc.wait(timeout=60) != 0:
                    raise RuntimeError(f"backend w{w.wid} exited with {w.proc.returncode}")
        finally:
            for w in self.workers:
                if w.proc.poll() is None:
                    w.proc.send_signal(signal.SIGKILL)
                    w.proc.wait()
        return self.hashes()

    def hashes(self) -> dict:
        out = {}
        path = os.path.join(self.workdir, "hashes.txt")
        if os.path.exists(path):
            for line in open(path):
                e, h = line.split()
                out[int(e)] = int(h)
        return out


# ----------------------------------------------------------- one process per GPU

def ring_fault_drill(eng, make_engine, join, rank: int, world: int, width: int, height: int, ckpt_dir: str, *,
                     seed: int = 0x5EED, victim: int = 3, kill_at: int = 25, gens: int = 50, every: int = 10,
                     topology: str = "torus"):
    """BASELINE.json config 5 in the form the multi-GPU bench runs it: the
    ranks of one job (one process per GPU, no supervisor) lose one of their
    backends mid-run and re-spawn its shard on a surviving GPU.

    Every rank seeds its shard and steps with fused hashes, all-reducing the
    partials into the global per-generation hashes and writing its shard
    checkpoint every `every` generations into `ckpt_dir` (a directory all
    ranks share).  After generation `kill_at` rank `victim` (capped at
    world - 1) drops its communicator and its context -- a backend lost
    between two steps, before it could checkpoint (the process itself stays
    alive, so the launcher does not tear the job down).  Then, as in
    ``BoardCreator.onCellTermination`` (BoardCreator.scala:120-154):

    * the survivors leave the old ring (gol_comm_abort);
    * the rank whose rows adjoin the lost block (the one above it; for rank 0
      the one below) restores the block's last checkpoint c <= kill_at, takes
      the kill_at - c rows above and below it at epoch c from the
      neighbours' checkpoint files (the light cone) and replays the block
      alone to kill_at (gol_replay; CellActor.scala:34,71-74,86 is the
      history replay it stands for), then holds its own rows and the lost
      ones as one context on its GPU -- nobody else rolls back;
    * the survivors join a new world - 1 rank ring (`join`, ranks renumbered
      in row order) and step on to `gens`.

    eng: this rank's context, already in the `world`-rank ring (rows of
    gol_shard_rows).  make_engine(row0, rows): a new context on this GPU.
    join(eng, tag, rank, world): put `eng` into the ring `tag`.

    Returns (the rank's context afterwards -- None for the lost rank, whose
    context is gone --, report).  The report holds the global hashes the
    caller checks: `before` (epochs 1..kill_at), `replayed` (epochs
    c + 1..kill_at: the replayed block's partials plus the survivors'),
    `at_recovery` (gol_hash over the new ring at kill_at), `after` (epochs
    kill_at + 1..gens) and `final` (gol_hash at gens), with wall times."""
    torus = topology == "torus"
    victim = max(0, min(victim, world - 1))
    host = victim - 1 if victim > 0 else 1
    row0, rows = shard_rows_py(height, rank, world)
    rep = {"victim_rank": victim, "host_rank": host, "world_before": world, "world_after": world - 1,
           "kill_at": kill_at, "generations": gens, "checkpoint_every": every}
    eng.seed(seed)
    epoch, before, parts = 0, [], {}
    my_file, ckpt_s = None, 0.0
    t_run = time.perf_counter()
    while epoch < kill_at:
        n = min(every - epoch % every, kill_at - epoch)
        part = eng.step(n, hashes=True)
        glob = eng.allreduce_u64(part)
        for k in range(n):
            parts[epoch + k + 1] = int(part[k])
        before.extend(int(x) for x in glob)
        epoch += n
        # a checkpoint every `every` generations; the lost rank dies right
        # after its last step, before it could write one
        if epoch % every == 0:
            t = time.perf_counter()
            wrote = not (rank == victim and epoch == kill_at)
            path = write_shard_checkpoint(ckpt_dir, eng.checkpoint()) if wrote else None
            # An epoch's checkpoint is complete once every rank has written
            # its file; only then may a rank drop its previous one.  A rank
            # lost at a checkpoint epoch (kill_at % every == 0) leaves that
            # epoch incomplete, so the previous files stay for its recovery.
            complete = int(eng.allreduce_u64(np.array([int(wrote)], dtype=np.uint64))[0]) == world
            if complete and my_file and my_file != path:
                os.unlink(my_file)
            if wrote and (complete or my_file is None):
                my_file = path
            ckpt_s += time.perf_counter() - t
    rep["before"] = before
    rep["checkpoint_s"] = round(ckpt_s, 3)
    rep["run_to_loss_s"] = round(time.perf_counter() - t_run, 3)
    if rank == victim:
        eng.comm_abort()
        eng.close()
        rep["role"] = "lost"
        return None, rep
    # -- recovery on the survivors
    t_loss = time.perf_counter()
    eng.comm_abort()
    new_rank, new_world = (rank if rank < victim else rank - 1), world - 1
    v0, vn = shard_rows_py(height, victim, world)
    c, hs = 0, None
    if rank == host:
        c = recovery_epoch(ckpt_dir, v0, v0 + vn, epoch, height, torus)
        d = epoch - c
        blob = assemble_checkpoint(ckpt_dir, c, v0, vn)
        above, below = light_cone(ckpt_dir, c, v0, vn, d, height, torus)
        h, _ = parse_checkpoint(blob)
        r = make_engine(v0, vn)
        try:
            r.restore(blob)
            hs = r.replay(d, above, below) if d else np.zeros(0, dtype=np.uint64)
            del blob
            lost_first = v0 + vn == row0  # the lost block lies above this one (victim 0, host 1)
            nrow0 = v0 if lost_first else row0
            merged, data = checkpoint_buffer(dict(h, row0=nrow0, epoch=epoch), rows + vn, h["wwords"])
            r.snapshot(out=data[:vn] if lost_first else data[rows:])
        finally:
            r.close()
        eng.snapshot(out=data[vn:] if lost_first else data[:rows])
        eng.close()
        row0, rows = nrow0, rows + vn
        eng = make_engine(row0, rows)
        eng.restore(merged)
        del merged, data
        rep["replay_s"] = round(time.perf_counter() - t_loss, 3)
    join(eng, "fault", new_rank, new_world)
    t_ready = time.perf_counter()
    # the checkpoint epoch the host replayed from, to every survivor
    c = int(eng.allreduce_u64(np.array([c], dtype=np.uint64))[0])
    mine = np.array([parts[e] for e in range(c + 1, epoch + 1)], dtype=np.uint64)
    if hs is not None:
        mine = mine + hs  # mod 2^64
    rep["checkpoint_epoch"] = c
    rep["replayed_generations"] = epoch - c
    rep["replayed"] = [int(x) for x in eng.allreduce_u64(mine)]
    rep["at_recovery"] = int(eng.allreduce_u64(np.array([eng.hash()], dtype=np.uint64))[0])
    rep["recovery_s"] = t_ready - t_loss  # this rank's; the caller takes the max
    rep["rows_after"] = [row0, rows]
    t1 = time.perf_counter()
    part = eng.step(gens - epoch, hashes=True) if gens > epoch else np.zeros(0, dtype=np.uint64)
    rep["after"] = [int(x) for x in eng.allreduce_u64(part)] if gens > epoch else []
    rep["after_s"] = time.perf_counter() - t1
    rep["final"] = int(eng.allreduce_u64(np.array([eng.hash()], dtype=np.uint64))[0])
    rep["role"] = "host" if rank == host else "survivor"
    return eng, rep


# ----------------------------------------------------------- CLI

def _parser():
    ap = argparse.ArgumentParser(prog="python -m gameoflife.elastic")
    sub = ap.add_subparsers(dest="cmd", required=True)
    w = sub.add_parser("worker", help="one backend process (started by the supervisor)")
    for name in ("--wid", "--width", "--height", "--every", "--seed", "--row0", "--rows", "--rank", "--world",
                 "--device", "--resume", "--target"):
        w.add_argument(name, type=int, required=True)
    for name in ("--ring-dir", "--workdir", "--ckpt-dir", "--topology", "--rule", "--shard"):
        w.add_argument(name, required=True)
    dm = sub.add_parser("demo", help="BASELINE.json config 5: kill backends mid-run")
    dm.add_argument("--width", type=int, default=262144)
    dm.add_argument("--height", type=int, default=262144)
    dm.add_argument("--gens", type=int, default=50)
    dm.add_argument("--every", type=int, default=10)
    dm.add_argument("--world", type=int, default=8)
    dm.add_argument("--kill", default="3@25", help="crash rank@generation, or 'none'")
    dm.add_argument("--workdir", default="/tmp/gol_elastic")
    dm.add_argument("--chunk", type=int, default=5, help="generations per supervisor release")
    dm.add_argument("--shard", default="gameoflife.elastic:GpuShard",
                    help="backend implementation module:Class (the CPU tests pass their oracle double)")
    return ap


def main(argv=None) -> int:
    a = _parser().parse_args(argv)
    if a.cmd == "worker":
        return worker_main(a)
    kill = None if a.kill == "none" else tuple(int(x) for x in a.kill.split("@"))
    sup = Supervisor(a.width, a.height, a.gens, a.world, a.workdir, a.every, kill=kill, chunk=a.chunk, shard=a.shard)
    got = sup.run()
    ref = Supervisor(a.width, a.height, a.gens, a.world, a.workdir + "_ref", a.every, chunk=a.chunk,
                     shard=a.shard).run()
    same = [got.get(e) == ref.get(e) for e in range(1, a.gens + 1)]
    print(json.dumps({"events": sup.events, "generations": a.gens, "hashes_equal": all(same)}))
    return 0 if all(same) else 1


if __name__ == "__main__":
    sys.exit(main())
