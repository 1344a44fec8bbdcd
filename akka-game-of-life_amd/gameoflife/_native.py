"""ctypes binding of libgol.so (include/gol.h).

The product path: every call goes to the HIP library.  If the library is not
built, importing this module raises immediately -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import re

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# GOL_LIB_PATH: an alternative build of the same library, for A/B timing
# experiments only (scripts/archive/ab_build.sh); products use the in-tree build.
LIB_PATH = os.environ.get("GOL_LIB_PATH") or os.path.join(PKG_ROOT, "lib", "libgol.so")
HEADER_PATH = os.path.join(os.path.dirname(PKG_ROOT), "include", "gol.h")

GOL_OK = 0
GOL_EINVAL = 1
GOL_EHIP = 2
GOL_ENOMEM = 3
GOL_ECOMM = 4
GOL_ESTATE = 5
GOL_ENODEV = 6

GOL_TORUS = 0
GOL_REF_CLIPPED = 1
GOL_UNIQUE_ID_BYTES = 128
# include/gol.h GOL_ABI_VERSION this binding is written against (2: the
# canonical state hash)
GOL_ABI_VERSION = 2


class GolError(RuntimeError):
    """A nonzero libgol return code (the analogue of the exception a cell
    actor throws, which the reference's supervisor turns into a Restart,
    BoardCreator.scala:42-45)."""

    def __init__(self, code: int, message: str):
        super().__init__(f"libgol error {code} ({_strerror(code)}): {message}")
        self.code = code
        self.message = message


class GolConfig(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int64),
        ("height", ctypes.c_int64),
        ("row0", ctypes.c_int64),
        ("rows", ctypes.c_int64),
        ("topology", ctypes.c_int32),
        ("birth_mask", ctypes.c_uint32),
        ("survive_mask", ctypes.c_uint32),
        ("device", ctypes.c_int32),
        ("vis_width", ctypes.c_int64),
        ("vis_height", ctypes.c_int64),
    ]


class GolProfileStats(ctypes.Structure):
    _fields_ = [
        ("kernel_ms", ctypes.c_double),
        ("launches", ctypes.c_uint64),
        ("generations", ctypes.c_uint64),
        ("exchange_ms", ctypes.c_double),
        ("exchanges", ctypes.c_uint64),
        ("boundary_ms", ctypes.c_double),
        ("boundary_launches", ctypes.c_uint64),
        ("halo_bytes_sent", ctypes.c_uint64),
        ("halo_bytes_received", ctypes.c_uint64),
        ("clock_ghz", ctypes.c_double),
        ("exchange_exposed_ms", ctypes.c_double),
        ("pass_tail_ms", ctypes.c_double),
    ]


class GolRuntimeInfo(ctypes.Structure):
    _fields_ = [
        ("abi_version", ctypes.c_int32),
        ("hip_runtime_version", ctypes.c_int32),
        ("hip_driver_version", ctypes.c_int32),
        ("rccl_version", ctypes.c_int32),
        ("hip_library", ctypes.c_char * 512),
        ("rccl_library", ctypes.c_char * 512),
        ("gol_library", ctypes.c_char * 512),
    ]


_c = ctypes
_vp = ctypes.c_void_p
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_u8p = ctypes.POINTER(ctypes.c_uint8)

_SIGNATURES = {
    "gol_abi_version": (_c.c_int, []),
    "gol_strerror": (_c.c_char_p, [_c.c_int]),
    "gol_last_error": (_c.c_char_p, [_vp]),
    "gol_device_count": (_c.c_int, [ctypes.POINTER(_c.c_int)]),
    "gol_shard_rows": (_c.c_int, [_c.c_int64, _c.c_int, _c.c_int, ctypes.POINTER(_c.c_int64),
                                  ctypes.POINTER(_c.c_int64)]),
    "gol_create": (_c.c_int, [ctypes.POINTER(_vp), ctypes.POINTER(GolConfig)]),
    "gol_destroy": (None, [_vp]),
    "gol_seed": (_c.c_int, [_vp, _c.c_uint64]),
    "gol_load": (_c.c_int, [_vp, _u32p, _c.c_int64]),
    "gol_step": (_c.c_int, [_vp, _c.c_uint32, _u64p]),
    "gol_step_ex": (_c.c_int, [_vp, _c.c_uint32, _u64p, _c.c_size_t]),
    "gol_epoch": (_c.c_int, [_vp, _u64p]),
    "gol_sync": (_c.c_int, [_vp]),
    "gol_hash": (_c.c_int, [_vp, _u64p]),
    "gol_snapshot": (_c.c_int, [_vp, _u32p, _c.c_int64]),
    "gol_profile_clock": (_c.c_int, [_vp, ctypes.POINTER(_c.c_double)]),
    "gol_snapshot_async": (_c.c_int, [_vp, _u32p, _c.c_int64]),
    "gol_checkpoint_async": (_c.c_int, [_vp, _vp, _c.c_size_t]),
    "gol_snapshot_wait": (_c.c_int, [_vp, _u64p]),
    "gol_snapshot_query": (_c.c_int, [_vp, ctypes.POINTER(_c.c_int)]),
    "gol_host_alloc": (_c.c_int, [_c.c_size_t, ctypes.POINTER(_vp)]),
    "gol_host_free": (None, [_vp]),
    "gol_get_cell": (_c.c_int, [_vp, _c.c_int64, _c.c_int64, ctypes.POINTER(_c.c_int)]),
    "gol_checkpoint_bytes": (_c.c_int, [_vp, ctypes.POINTER(_c.c_size_t)]),
    "gol_checkpoint": (_c.c_int, [_vp, _vp, _c.c_size_t]),
    "gol_restore": (_c.c_int, [_vp, _vp, _c.c_size_t]),
    "gol_comm_unique_id": (_c.c_int, [_u8p]),
    "gol_comm_init": (_c.c_int, [_vp, _u8p, _c.c_int, _c.c_int]),
    "gol_comm_allreduce_u64": (_c.c_int, [_vp, _u64p, _c.c_uint32]),
    "gol_comm_abort": (_c.c_int, [_vp]),
    "gol_comm_init_loopback": (_c.c_int, [_vp, _c.c_char_p, _c.c_int, _c.c_int]),
    "gol_replay": (_c.c_int, [_vp, _c.c_uint32, _u32p, _u32p, _c.c_int64, _u64p]),
    "gol_profile_enable": (_c.c_int, [_vp, _c.c_int]),
    "gol_profile_read": (_c.c_int, [_vp, ctypes.POINTER(_c.c_double), _u64p, _u64p]),
    "gol_profile_reset": (_c.c_int, [_vp]),
    "gol_set_tuning": (_c.c_int, [_vp, _c.c_int32, _c.c_int32, _c.c_int32]),
    "gol_selftest": (_c.c_int, [_c.c_int, _u32p]),
    "gol_occupancy": (_c.c_int, [_vp, _c.c_int32, ctypes.POINTER(_c.c_int32), ctypes.POINTER(_c.c_int32)]),
    "gol_pass_plan": (_c.c_int, [_vp, _c.c_uint32, _c.c_int32, ctypes.POINTER(_c.c_int32), _c.c_int32,
                                 ctypes.POINTER(_c.c_int32)]),
    "gol_group_create": (_c.c_int, [ctypes.POINTER(_vp), ctypes.POINTER(_vp), _c.c_int]),
    "gol_group_step": (_c.c_int, [_vp, _c.c_uint32, _u64p]),
    "gol_group_step_partials": (_c.c_int, [_vp, _c.c_uint32, _u64p, _u64p]),
    "gol_group_sync": (_c.c_int, [_vp]),
    "gol_group_last_error": (_c.c_char_p, [_vp]),
    "gol_group_destroy": (None, [_vp]),
    "gol_diag_take_hip_error": (_c.c_int, [ctypes.POINTER(_c.c_int)]),
    "gol_diag_absorbed": (_c.c_int, [_u64p, _c.c_char_p, _c.c_size_t]),
    "gol_profile_stats_read": (_c.c_int, [_vp, ctypes.POINTER(GolProfileStats)]),
    "gol_runtime_info_get": (_c.c_int, [ctypes.POINTER(GolRuntimeInfo)]),
    "gol_device_layout": (_c.c_int, [_c.c_int32, _c.c_int64, ctypes.POINTER(_c.c_int32)]),
}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libgol.so not found at {LIB_PATH}; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (there is no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.gol_abi_version() != GOL_ABI_VERSION:
        raise ImportError(f"{LIB_PATH} has ABI version {lib.gol_abi_version()}, this binding needs "
                          f"{GOL_ABI_VERSION}; rebuild it")
    return lib


lib = _load()


def _strerror(code: int) -> str:
    return lib.gol_strerror(code).decode()


def check(code: int, ctx=None) -> None:
    if code != GOL_OK:
        msg = lib.gol_last_error(ctx)
        raise GolError(code, msg.decode() if msg else "")


def header_symbols(path: str = HEADER_PATH) -> list[str]:
    """Names of the functions declared in include/gol.h."""
    text = open(path).read()
    return sorted(set(re.findall(r"^\s*(?:[A-Za-z_][\w\s\*]*?)\b(gol_\w+)\s*\(", text, re.M)))


def device_count() -> int:
    n = ctypes.c_int(0)
    check(lib.gol_device_count(ctypes.byref(n)))
    return n.value


def device_ilv(width: int, topology: int = GOL_TORUS) -> int:
    """Words per interleave group of libgol's device layout (gol_capi.cpp
    device_ilv, a function of the geometry alone): a torus whose rows hold
    whole pairs of 32-bit words is pair-interleaved (2), any other board
    row-major (1).  Informational: host buffers are row-major and the state
    hash is defined over the cells."""
    ww = (width + 31) // 32
    if topology != GOL_TORUS:
        return 1
    return 2 if ww % 2 == 0 else 1


def device_layout(width: int, topology: int = GOL_TORUS) -> int:
    """libgol's own answer (gol_device_layout) -- device_ilv restates it."""
    k = ctypes.c_int32(0)
    check(lib.gol_device_layout(topology, width, ctypes.byref(k)))
    return k.value


def shard_rows(height: int, rank: int, nranks: int) -> tuple[int, int]:
    r0, rows = ctypes.c_int64(0), ctypes.c_int64(0)
    check(lib.gol_shard_rows(height, rank, nranks, ctypes.byref(r0), ctypes.byref(rows)))
    return r0.value, rows.value


def unique_id() -> bytes:
    buf = (ctypes.c_uint8 * GOL_UNIQUE_ID_BYTES)()
    check(lib.gol_comm_unique_id(buf))
    return bytes(buf)


def take_hip_error() -> int:
    """The calling thread's pending HIP status (0: none), taken off the
    thread (gol_diag_take_hip_error)."""
    c = ctypes.c_int(0)
    check(lib.gol_diag_take_hip_error(ctypes.byref(c)))
    return c.value


def absorbed() -> tuple[int, str]:
    """(count, last description) of the HIP statuses RCCL calls left behind
    and libgol absorbed (gol_diag_absorbed)."""
    n = ctypes.c_uint64(0)
    buf = ctypes.create_string_buffer(256)
    check(lib.gol_diag_absorbed(ctypes.byref(n), buf, len(buf)))
    return n.value, buf.value.decode()


def _version(v: int, major_div: int, minor_div: int) -> str:
    return f"{v // major_div}.{v % major_div // minor_div}.{v % minor_div}" if v else "unknown"


def runtime_info() -> dict:
    """The HIP runtime and RCCL this process's libgol is bound to, and the
    files they were loaded from (gol_runtime_info_get; host-only)."""
    ri = GolRuntimeInfo()
    check(lib.gol_runtime_info_get(ctypes.byref(ri)))
    return {"hip_runtime_version": ri.hip_runtime_version,
            "hip_runtime": _version(ri.hip_runtime_version, 10_000_000, 100_000),
            "hip_driver_version": ri.hip_driver_version,
            "rccl_version": ri.rccl_version,
            "rccl": _version(ri.rccl_version, 10_000, 100),
            "hip_library": ri.hip_library.decode(errors="replace"),
            "rccl_library": ri.rccl_library.decode(errors="replace"),
            "gol_library": ri.gol_library.decode(errors="replace"),
            "torch_loaded": "torch" in __import__("sys").modules}
