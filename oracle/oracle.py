"""CPU oracle for the generation step -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import this module, and only as the checker (or as the timed
CPU baseline).  The product path (``libgol.so`` via ``gameoflife``) never
imports it.

PARITY UNPINNED: the reference ships no tests/fixtures and cannot be built or
run here (no JVM/sbt/Akka, no network).  Two
independent restatements are kept and cross-checked against each other and
against hand-derived known-answer patterns:

* ``liboracle.so`` (``gol_oracle.c``): scalar per-cell step (the literal
  restatement of package.scala:17-28 + NextStateCellGathererActor.scala:39-46)
  plus a bit-packed multithreaded step (also the CPU baseline);
* ``np_step`` below: a numpy restatement written separately from the C one.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

TORUS = 0
REF_CLIPPED = 1
MODE_MASKS = 0
MODE_REF_EFFECTIVE = 1

LIFE = (0x008, 0x00C)          # B3/S23 (BASELINE.json north_star)
REF_LITERAL = (0x000, 0x1F7)   # NextStateCellGathererActor.scala:44 with a multiset count
REF_EFFECTIVE = (0x000, 0x1FF)  # what :42-44 actually computes (Set collapse) == identity

_u32p = ctypes.POINTER(ctypes.c_uint32)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_i64 = ctypes.c_int64

_lib = None


def build(force: bool = False) -> str:
    """Compile liboracle.so with the committed Makefile (gcc, OpenMP)."""
    if force or not os.path.exists(LIB_PATH) or (
        os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "gol_oracle.c"))
    ):
        subprocess.run(["make", "-C", HERE, "-B" if force else "all"], check=True,
                       stdout=subprocess.DEVNULL)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_splitmix64.restype = ctypes.c_uint64
        L.oracle_splitmix64.argtypes = [ctypes.c_uint64]
        L.oracle_seed_packed.argtypes = [_u32p, _i64, _i64, _i64, _i64, ctypes.c_uint64]
        L.oracle_java_random_cells.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int64]
        L.oracle_step_cells.argtypes = [_u8p, _u8p, _i64, _i64, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_uint32, ctypes.c_uint32, _i64, _i64]
        L.oracle_step_packed.argtypes = [_u32p, _u32p, _i64, _i64, _i64, ctypes.c_int,
                                         ctypes.c_uint32, ctypes.c_uint32, _i64, _i64, ctypes.c_int]
        L.oracle_hash_packed.restype = ctypes.c_uint64
        L.oracle_hash_packed.argtypes = [_u32p, _i64, _i64, _i64, _i64]
        L.oracle_canonical_words.argtypes = [_u32p, _i64, _i64, _u32p, _u32p]
        L.oracle_hash_row_key.restype = ctypes.c_uint32
        L.oracle_hash_row_key.argtypes = [_i64, ctypes.c_int]
        L.oracle_hash_pair_key.restype = ctypes.c_uint32
        L.oracle_hash_pair_key.argtypes = [ctypes.c_uint32]
        L.oracle_run_packed.argtypes = [_u32p, _u32p, _i64, _i64, _i64, ctypes.c_int,
                                        ctypes.c_uint32, ctypes.c_uint32, _i64, _i64, _i64,
                                        _u64p, ctypes.c_int]
        L.oracle_pack.argtypes = [_u8p, _u32p, _i64, _i64, _i64]
        L.oracle_unpack.argtypes = [_u32p, _u8p, _i64, _i64, _i64]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


def wwords(W: int) -> int:
    return (W + 31) // 32


# ---------------------------------------------------------------- boards

def seed_packed(W: int, H: int, seed: int = 0x5EED, row0: int = 0, rows: int | None = None,
                pitch: int | None = None) -> np.ndarray:
    rows = H if rows is None else rows
    pitch = wwords(W) if pitch is None else pitch
    out = np.zeros((rows, pitch), dtype=np.uint32)
    lib().oracle_seed_packed(_p(out, _u32p), W, row0, rows, pitch, seed)
    return out


def java_random_cells(w: int, h: int, seed: int) -> np.ndarray:
    """(h+1) x (w+1) uint8 board, java.util.Random(seed) in BoardCreator order."""
    out = np.zeros((h + 1, w + 1), dtype=np.uint8)
    lib().oracle_java_random_cells(_p(out, _u8p), w, h, seed)
    return out


def pack(cells: np.ndarray, pitch: int | None = None) -> np.ndarray:
    H, W = cells.shape
    pitch = wwords(W) if pitch is None else pitch
    cells = np.ascontiguousarray(cells, dtype=np.uint8)
    out = np.zeros((H, pitch), dtype=np.uint32)
    lib().oracle_pack(_p(cells, _u8p), _p(out, _u32p), W, H, pitch)
    return out


def unpack(packed: np.ndarray, W: int) -> np.ndarray:
    packed = np.ascontiguousarray(packed, dtype=np.uint32)
    H, pitch = packed.shape
    out = np.zeros((H, W), dtype=np.uint8)
    lib().oracle_unpack(_p(packed, _u32p), _p(out, _u8p), W, H, pitch)
    return out


# ---------------------------------------------------------------- steps

def step_cells(cells: np.ndarray, topology: int = TORUS, rule=LIFE, mode: int = MODE_MASKS,
               vis: tuple[int, int] | None = None) -> np.ndarray:
    H, W = cells.shape
    vw, vh = vis if vis is not None else ((W - 1, H - 1) if topology == REF_CLIPPED else (W, H))
    cur = np.ascontiguousarray(cells, dtype=np.uint8)
    nxt = np.zeros_like(cur)
    lib().oracle_step_cells(_p(cur, _u8p), _p(nxt, _u8p), W, H, topology, mode,
                            rule[0], rule[1], vw, vh)
    return nxt


def step_packed(packed: np.ndarray, W: int, topology: int = TORUS, rule=LIFE,
                vis: tuple[int, int] | None = None, nthreads: int = 0) -> np.ndarray:
    packed = np.ascontiguousarray(packed, dtype=np.uint32)
    H, pitch = packed.shape
    vw, vh = vis if vis is not None else ((W - 1, H - 1) if topology == REF_CLIPPED else (W, H))
    out = np.zeros_like(packed)
    lib().oracle_step_packed(_p(packed, _u32p), _p(out, _u32p), W, H, pitch, topology,
                             rule[0], rule[1], vw, vh, nthreads)
    return out


def run_packed(packed: np.ndarray, W: int, gens: int, topology: int = TORUS, rule=LIFE,
               vis: tuple[int, int] | None = None, nthreads: int = 0,
               want_hashes: bool = True):
    """Run `gens` generations; returns (final board, per-generation hashes)."""
    board = np.ascontiguousarray(packed, dtype=np.uint32).copy()
    H, pitch = board.shape
    vw, vh = vis if vis is not None else ((W - 1, H - 1) if topology == REF_CLIPPED else (W, H))
    tmp = np.zeros_like(board)
    hashes = np.zeros(gens, dtype=np.uint64) if want_hashes else None
    lib().oracle_run_packed(_p(board, _u32p), _p(tmp, _u32p), W, H, pitch, topology,
                            rule[0], rule[1], vw, vh, gens,
                            _p(hashes, _u64p) if want_hashes else None, nthreads)
    return board, hashes


def hash_packed(packed: np.ndarray, W: int, row0: int = 0, topology: int = TORUS) -> int:
    """State hash of row-major packed rows [row0, row0 + rows) of a board: a
    function of the cells alone, so `topology` does not
    enter it (kept for the callers that pass it)."""
    del topology
    packed = np.ascontiguousarray(packed, dtype=np.uint32)
    rows, pitch = packed.shape
    return int(lib().oracle_hash_packed(_p(packed, _u32p), wwords(W), row0, rows, pitch))


# ------------------------------------------------- independent numpy restatement

def np_canonical_words(packed: np.ndarray, W: int) -> np.ndarray:
    """Row-major packed rows -> the hash's canonical words (independent numpy
    restatement): column 64 g + 2 b + j -> bit b of word 2 g + j, the row
    padded with dead columns to whole 64-column groups."""
    ww = wwords(W)
    p = np.asarray(packed, dtype=np.uint32)[:, :ww]
    if ww % 2:
        p = np.concatenate([p, np.zeros((p.shape[0], 1), dtype=np.uint32)], axis=1)
    rows, nw = p.shape
    bits = ((p[:, :, None] >> np.arange(32, dtype=np.uint32)) & 1).reshape(rows, nw // 2, 64)
    weights = np.uint64(1) << np.arange(32, dtype=np.uint64)
    out = np.empty((rows, nw), dtype=np.uint32)
    for j in range(2):
        out[:, j::2] = (bits[:, :, j::2].astype(np.uint64) * weights).sum(axis=2).astype(np.uint32)
    return out


def np_hash(packed: np.ndarray, W: int, row0: int = 0, topology: int = TORUS) -> int:
    """Same hash spec as gol_oracle.c (DESIGN.md "State hash"), written
    independently with numpy: sum of w * A(y, c % 2) * B(c / 2) mod 2^64 over
    the canonical words w (np_canonical_words)."""
    del topology
    grp = 2
    p = np_canonical_words(packed, W).astype(np.uint64)
    rows, ww = p.shape
    m32 = np.uint64(0xFFFFFFFF)
    with np.errstate(over="ignore"):
        y = np.arange(rows, dtype=np.uint64) + np.uint64(row0)
        t = (y * np.uint64(0x9E3779B1)) & m32
        a0 = ((((t ^ (t >> np.uint64(15))) << np.uint64(1)) | np.uint64(1)) & m32)
        k = np.arange(ww, dtype=np.uint64) // np.uint64(grp)
        h = (k + np.uint64(0x7F4A7C15)) & m32
        h ^= h >> np.uint64(16)
        h = (h * np.uint64(0x85EBCA6B)) & m32
        h ^= h >> np.uint64(13)
        h = (h * np.uint64(0xC2B2AE35)) & m32
        h ^= h >> np.uint64(16)
        b = h | np.uint64(1)
        ph = (np.arange(ww, dtype=np.uint64) % np.uint64(grp))
        a = (a0[:, None] + ph[None, :] * np.uint64(0x6A09E666)) & m32
        terms = p * (a * b[None, :])
        return int(terms.sum(dtype=np.uint64))


def np_step(cells: np.ndarray, topology: int = TORUS, rule=LIFE, mode: int = MODE_MASKS,
            vis: tuple[int, int] | None = None) -> np.ndarray:
    """numpy restatement: np.roll for the torus, zero-padded slicing for the
    reference's clipped geometry (package.scala:17-28)."""
    c = np.asarray(cells, dtype=np.int32)
    H, W = c.shape
    if topology == TORUS:
        n = sum(np.roll(np.roll(c, dy, 0), dx, 1)
                for dy in (-1, 0, 1) for dx in (-1, 0, 1) if (dx, dy) != (0, 0))
    else:
        vw, vh = vis if vis is not None else (W - 1, H - 1)
        v = np.zeros((H + 2, W + 2), dtype=np.int32)
        v[1:1 + min(vh, H), 1:1 + min(vw, W)] = c[:min(vh, H), :min(vw, W)]
        n = sum(v[1 + dy:1 + dy + H, 1 + dx:1 + dx + W]
                for dy in (-1, 0, 1) for dx in (-1, 0, 1) if (dx, dy) != (0, 0))
    if mode == MODE_REF_EFFECTIVE:
        any_alive = (n > 0).astype(np.int32)  # Set[Boolean] collapse
        return np.where((c == 1) & (any_alive == 3), 1 - c, c).astype(np.uint8)
    birth = np.array([(rule[0] >> k) & 1 for k in range(9)], dtype=np.uint8)
    survive = np.array([(rule[1] >> k) & 1 for k in range(9)], dtype=np.uint8)
    return np.where(c == 1, survive[n], birth[n]).astype(np.uint8)


def np_seed(W: int, H: int, seed: int = 0x5EED) -> np.ndarray:
    """Independent numpy restatement of the splitmix64 board seeding."""
    ww = wwords(W)
    i = np.arange(H * ww, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + np.uint64(0x9E3779B97F4A7C15) * (i + np.uint64(1))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    words = (z >> np.uint64(32)).astype(np.uint32).reshape(H, ww)
    if W % 32:
        words[:, -1] &= np.uint32((1 << (W % 32)) - 1)
    return words


def java_random_next_booleans(seed: int, n: int) -> list[bool]:
    """Pure-Python java.util.Random(seed).nextBoolean() x n (small n only)."""
    mask = (1 << 48) - 1
    s = (seed ^ 0x5DEECE66D) & mask
    out = []
    for _ in range(n):
        s = (s * 0x5DEECE66D + 0xB) & mask
        out.append((s >> 47) != 0)
    return out


def reference_commit_epochs(w: int, h: int, target: int) -> dict:
    """The epoch each cell of the reference's (w+1) x (h+1) board has
    committed once every message has been delivered, capped at `target`:
    a restatement of the reference's commit condition, not of its rule.

    A cell at epoch e spawns a gatherer that asks every visible neighbour
    (package.scala:17-28) for its state at epoch e
    (NextStateCellGathererActor.scala:26-27,32-36); a neighbour answers once it
    holds epoch e, from its never-pruned history, and queues the request until
    then (CellActor.scala:71-77).  The gatherer completes -- and the cell
    commits e + 1 (:39-47, CellActor.scala:79-89) -- only when the last
    expected answer arrives, so a cell with no visible neighbour never commits
    (its gatherer retries, fails, and the cell re-asks for neighbours forever:
    :49-53, CellActor.scala:92-94), and its neighbours stop one epoch after it.
    Returns {(x, y): epoch}."""
    cells = [(i, j) for i in range(w + 1) for j in range(h + 1)]
    nbrs = {c: [(c[0] + di, c[1] + dj) for di in (-1, 0, 1) for dj in (-1, 0, 1)
                if (di, dj) != (0, 0) and 0 <= c[0] + di < w and 0 <= c[1] + dj < h] for c in cells}
    epoch = {c: 0 for c in cells}
    changed = True
    while changed:
        changed = False
        for c in cells:
            e = epoch[c]
            if e < target and nbrs[c] and all(epoch[n] >= e for n in nbrs[c]):
                epoch[c] = e + 1
                changed = True
    return epoch


def reference_completes(w: int, h: int, generations: int = 3) -> bool:
    """Does the reference board of size (w, h) reach `generations` whole
    generations (every cell committed)?  See reference_commit_epochs."""
    return min(reference_commit_epochs(w, h, generations).values()) >= generations
