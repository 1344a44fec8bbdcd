"""Shard engine: one libgol context = one backend worker owning a row block.

The reference's backend hosts cell actors (CellActor.scala:10-102), each
holding its own history and computing its next state by messaging its
neighbours.  Here a backend worker owns a contiguous row block of the board in
HBM and advances all of it per generation through libgol.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N
from .rules import Rule, rule_by_name


class GolEngine:
    """A shard context on one GPU (gol_create .. gol_destroy)."""

    def __init__(self, width: int, height: int, *, topology: str = "torus",
                 rule: Rule | str = "life", device: int = 0, row0: int = 0,
                 rows: int | None = None, vis: tuple[int, int] | None = None):
        self.rule = rule_by_name(rule) if isinstance(rule, str) else rule
        self.topology = topology
        topo = {"torus": N.GOL_TORUS, "ref-clipped": N.GOL_REF_CLIPPED}[topology]
        cfg = N.GolConfig()
        cfg.width = width
        cfg.height = height
        cfg.row0 = row0
        cfg.rows = (height - row0) if rows is None else rows
        cfg.topology = topo
        cfg.birth_mask = self.rule.birth
        cfg.survive_mask = self.rule.survive
        cfg.device = device
        cfg.vis_width, cfg.vis_height = vis if vis is not None else (0, 0)
        h = ctypes.c_void_p()
        N.check(N.lib.gol_create(ctypes.byref(h), ctypes.byref(cfg)))
        self._h = h
        self.width, self.height = width, height
        self.row0, self.rows = row0, cfg.rows
        self.wwords = (width + 31) // 32
        self.device = device

    # -- lifecycle ---------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            N.lib.gol_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc: int) -> None:
        N.check(rc, self._h)

    # -- state -------------------------------------------------------------
    def seed(self, seed: int = 0x5EED) -> None:
        self._chk(N.lib.gol_seed(self._h, seed))

    def load(self, packed: np.ndarray) -> None:
        a = np.ascontiguousarray(packed, dtype=np.uint32)
        assert a.shape[0] == self.rows and a.shape[1] >= self.wwords, a.shape
        self._chk(N.lib.gol_load(self._h, a.ctypes.data_as(N._u32p), a.shape[1]))

    def snapshot(self, out: np.ndarray | None = None) -> np.ndarray:
        """Current board, row-major host layout.  `out`: a caller-owned
        (rows, wwords) uint32 C-contiguous buffer to fill -- reusing one (or a
        pinned one) avoids first-touch page faults on every snapshot."""
        if out is None:
            out = np.zeros((self.rows, self.wwords), dtype=np.uint32)
        elif out.dtype != np.uint32 or out.shape != (self.rows, self.wwords) or not out.flags.c_contiguous:
            raise ValueError(f"snapshot buffer must be a C-contiguous uint32 array of shape {(self.rows, self.wwords)}")
        self._chk(N.lib.gol_snapshot(self._h, out.ctypes.data_as(N._u32p), self.wwords))
        return out

    def snapshot_async(self, out: np.ndarray) -> None:
        """Start copying the current board into `out` (as snapshot()'s
        buffer; a page-locked one from host_buffer() keeps the call from
        blocking) while later steps run; snapshot_wait() finishes it."""
        if out.dtype != np.uint32 or out.shape != (self.rows, self.wwords) or not out.flags.c_contiguous:
            raise ValueError(f"snapshot buffer must be a C-contiguous uint32 array of shape {(self.rows, self.wwords)}")
        self._chk(N.lib.gol_snapshot_async(self._h, out.ctypes.data_as(N._u32p), self.wwords))
        self._snap_out = out  # keep the buffer alive while the copy is in flight

    def snapshot_wait(self) -> int:
        """Finish the snapshot started by snapshot_async; returns its epoch."""
        e = ctypes.c_uint64(0)
        try:
            self._chk(N.lib.gol_snapshot_wait(self._h, ctypes.byref(e)))
        finally:
            self._snap_out = None
        return e.value

    def snapshot_landed(self) -> bool:
        """Has the snapshot started by snapshot_async reached its buffer?
        (gol_snapshot_query: non-blocking; snapshot_wait still ends it)."""
        d = ctypes.c_int(0)
        self._chk(N.lib.gol_snapshot_query(self._h, ctypes.byref(d)))
        return bool(d.value)

    def host_buffer(self) -> np.ndarray:
        """A page-locked (rows, wwords) uint32 buffer for snapshots / loads."""
        return host_array((self.rows, self.wwords))

    def step(self, generations: int = 1, hashes: bool = False):
        """Advance; returns the per-generation partial hashes (uint64) if asked."""
        if hashes:
            out = np.zeros(generations, dtype=np.uint64)
            self._chk(N.lib.gol_step_ex(self._h, generations, out.ctypes.data_as(N._u64p), out.size))
            return out
        self._chk(N.lib.gol_step(self._h, generations, None))
        return None

    def sync(self) -> None:
        self._chk(N.lib.gol_sync(self._h))

    @property
    def epoch(self) -> int:
        e = ctypes.c_uint64(0)
        self._chk(N.lib.gol_epoch(self._h, ctypes.byref(e)))
        return e.value

    def hash(self) -> int:
        h = ctypes.c_uint64(0)
        self._chk(N.lib.gol_hash(self._h, ctypes.byref(h)))
        return h.value

    def get_cell(self, x: int, y: int) -> bool:
        s = ctypes.c_int(0)
        self._chk(N.lib.gol_get_cell(self._h, x, y, ctypes.byref(s)))
        return bool(s.value)

    def checkpoint(self) -> np.ndarray:
        """gol_checkpoint into a new uint8 array (a bytes-like buffer: file
        writes, parse_checkpoint and restore take it as is).  No zero-fill and
        no bytes copy: at 0.5 GiB per shard that was ~0.3 s per checkpoint."""
        n = self.checkpoint_bytes()
        out = np.empty(n, dtype=np.uint8)
        self._chk(N.lib.gol_checkpoint(self._h, out.ctypes.data_as(ctypes.c_void_p), n))
        return out

    def checkpoint_bytes(self) -> int:
        n = ctypes.c_size_t(0)
        self._chk(N.lib.gol_checkpoint_bytes(self._h, ctypes.byref(n)))
        return n.value

    def checkpoint_async(self, out: np.ndarray) -> None:
        """Start a checkpoint into `out` (uint8, checkpoint_bytes() long; a
        page-locked one from host_array keeps the call from blocking); finish
        it with snapshot_wait()."""
        if out.dtype != np.uint8 or out.size < self.checkpoint_bytes() or not out.flags.c_contiguous:
            raise ValueError("checkpoint buffer must be a C-contiguous uint8 array of checkpoint_bytes()")
        self._chk(N.lib.gol_checkpoint_async(self._h, out.ctypes.data_as(ctypes.c_void_p), out.size))
        self._snap_out = out

    def restore(self, blob) -> None:
        """Restore a checkpoint (bytes, or any buffer such as a uint8 array)."""
        arr = np.frombuffer(blob, dtype=np.uint8)
        self._chk(N.lib.gol_restore(self._h, arr.ctypes.data_as(ctypes.c_void_p), arr.size))

    # -- multi-GPU -----------------------------------------------------------
    def comm_init(self, uid: bytes, rank: int, nranks: int) -> None:
        arr = (ctypes.c_uint8 * N.GOL_UNIQUE_ID_BYTES).from_buffer_copy(uid)
        self._chk(N.lib.gol_comm_init(self._h, arr, rank, nranks))

    def comm_init_loopback(self, key: str, rank: int, nranks: int) -> None:
        """Join the in-process loopback ring `key` (gol_comm_init_loopback, a
        test transport running the RCCL schedule's exact halo operations
        between contexts of this process, one thread each)."""
        self._chk(N.lib.gol_comm_init_loopback(self._h, key.encode(), rank, nranks))

    def comm_abort(self) -> None:
        """Leave the ring (gol_comm_abort); comm_init may join a new one."""
        self._chk(N.lib.gol_comm_abort(self._h))

    def replay(self, generations: int, above: np.ndarray, below: np.ndarray, hashes: bool = True):
        """Light-cone replay (gol_replay): advance this shard `generations`
        generations alone from the `generations` rows above and below it at
        its current epoch.  Returns the shard's per-generation partial hashes."""
        a = np.ascontiguousarray(above, dtype=np.uint32)
        b = np.ascontiguousarray(below, dtype=np.uint32)
        if a.shape != (generations, self.wwords) or b.shape != a.shape:
            raise ValueError(f"light-cone rows must be ({generations}, {self.wwords}) arrays")
        out = np.zeros(generations, dtype=np.uint64) if hashes else None
        self._chk(N.lib.gol_replay(self._h, generations, a.ctypes.data_as(N._u32p), b.ctypes.data_as(N._u32p),
                                   self.wwords, out.ctypes.data_as(N._u64p) if hashes else None))
        return out

    def allreduce_u64(self, values: np.ndarray) -> np.ndarray:
        v = np.ascontiguousarray(values, dtype=np.uint64).copy()
        self._chk(N.lib.gol_comm_allreduce_u64(self._h, v.ctypes.data_as(N._u64p), v.size))
        return v

    # -- timing / tuning -----------------------------------------------------
    def profile(self, enable: bool = True) -> None:
        self._chk(N.lib.gol_profile_enable(self._h, 1 if enable else 0))

    def profile_read(self) -> tuple[float, int, int]:
        """(kernel ms, launches, generations advanced by those launches)."""
        ms, n, g = ctypes.c_double(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
        self._chk(N.lib.gol_profile_read(self._h, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(g)))
        return ms.value, n.value, g.value

    def profile_reset(self) -> None:
        self._chk(N.lib.gol_profile_reset(self._h))

    def profile_clock(self) -> float:
        """GHz the GPU held during the profiled launches since the reset
        (in-kernel clock probe, gol_profile_clock); 0.0 if none."""
        g = ctypes.c_double(0)
        self._chk(N.lib.gol_profile_clock(self._h, ctypes.byref(g)))
        return g.value

    def profile_stats(self) -> dict:
        """gol_profile_stats_read: the profiled passes since the reset split
        into the dominant launch, the halo exchange on the comm stream and the
        boundary launches, with the halo bytes posted to the ring."""
        st = N.GolProfileStats()
        self._chk(N.lib.gol_profile_stats_read(self._h, ctypes.byref(st)))
        return {k: getattr(st, k) for k, _ in N.GolProfileStats._fields_}

    def occupancy(self, gens_per_pass: int) -> tuple[int, int]:
        """(resident waves per CU, strip width in words) of a G-generation pass."""
        w, s = ctypes.c_int32(0), ctypes.c_int32(0)
        self._chk(N.lib.gol_occupancy(self._h, gens_per_pass, ctypes.byref(w), ctypes.byref(s)))
        return w.value, s.value

    def pass_plan(self, generations: int, hashes: bool = False) -> list[int]:
        """Pass depths gol_step would use for `generations` (<= 1024) generations."""
        buf = (ctypes.c_int32 * max(generations, 1))()
        n = ctypes.c_int32(0)
        self._chk(N.lib.gol_pass_plan(self._h, generations, int(hashes), buf, len(buf), ctypes.byref(n)))
        return list(buf[:n.value])

    def set_tuning(self, band_rows: int = 0, gens_per_pass: int = 0, words_per_lane: int = 0) -> None:
        """Performance knobs only (gol_set_tuning): rows per band, generations
        per HBM pass (1..12), words per lane (1/2/4, 0 = auto)."""
        self._chk(N.lib.gol_set_tuning(self._h, band_rows, gens_per_pass, words_per_lane))


class ShardGroup:
    """In-process group of shard engines of one board (gol_group_*): stepped
    in lockstep with device-to-device halo copies.  Engines must be given in
    row order and cover the board; they stay owned by the caller."""

    def __init__(self, shards: list[GolEngine]):
        self.shards = list(shards)
        arr = (ctypes.c_void_p * len(shards))(*[s._h.value for s in shards])
        h = ctypes.c_void_p()
        N.check(N.lib.gol_group_create(ctypes.byref(h), arr, len(shards)))
        self._h = h

    def _chk(self, rc: int) -> None:
        if rc != N.GOL_OK:
            raise N.GolError(rc, (N.lib.gol_group_last_error(self._h) or b"").decode())

    def step(self, generations: int = 1, hashes: bool = False, partials: bool = False):
        """Advance every shard; returns the global per-generation hashes if
        asked, and with partials=True also every shard's partials as a
        (shards, generations) array (gol_group_step_partials)."""
        if partials:
            out = np.zeros(generations, dtype=np.uint64)
            part = np.zeros((len(self.shards), generations), dtype=np.uint64)
            self._chk(N.lib.gol_group_step_partials(self._h, generations, out.ctypes.data_as(N._u64p),
                                                    part.ctypes.data_as(N._u64p)))
            return out, part
        if hashes:
            out = np.zeros(generations, dtype=np.uint64)
            self._chk(N.lib.gol_group_step(self._h, generations, out.ctypes.data_as(N._u64p)))
            return out
        self._chk(N.lib.gol_group_step(self._h, generations, None))
        return None

    def sync(self) -> None:
        self._chk(N.lib.gol_group_sync(self._h))

    @property
    def epoch(self) -> int:
        return self.shards[0].epoch

    def snapshot(self) -> np.ndarray:
        return np.vstack([s.snapshot() for s in self.shards])

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            N.lib.gol_group_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _HostBlock:
    """Owner of one gol_host_alloc block; freed when the last array viewing
    it is garbage-collected."""

    def __init__(self, nbytes: int):
        self.ptr = ctypes.c_void_p()
        N.check(N.lib.gol_host_alloc(nbytes, ctypes.byref(self.ptr)))

    def __del__(self):
        try:
            if getattr(self, "ptr", None) is not None and self.ptr.value:
                N.lib.gol_host_free(self.ptr)
                self.ptr = None
        except Exception:  # interpreter shutdown: the library may be gone already
            pass


def host_array(shape, dtype=np.uint32) -> np.ndarray:
    """A numpy array over page-locked host memory (gol_host_alloc); the block
    is freed when the array (and every view of it) is garbage-collected."""
    dt = np.dtype(dtype)
    nbytes = int(np.prod(shape)) * dt.itemsize
    block = _HostBlock(max(1, nbytes))
    buf = (ctypes.c_char * max(1, nbytes)).from_address(block.ptr.value)
    buf._gol_block = block  # array -> buf -> block
    return np.frombuffer(buf, dtype=dt, count=int(np.prod(shape))).reshape(shape)


def selftest(device: int = 0) -> np.ndarray:
    rep = np.zeros(256, dtype=np.uint32)
    N.check(N.lib.gol_selftest(device, rep.ctypes.data_as(N._u32p)))
    return rep
