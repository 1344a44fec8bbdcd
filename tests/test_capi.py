"""CPU tests of the C-ABI boundary: libgol.so loads, exports every symbol
include/gol.h declares, its pure-host entry points behave, and the product
path refuses to run without a HIP device (no CPU fallback)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from gameoflife import _native as N
from gameoflife import codec
from gameoflife.shard import shard_rows_py
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_exports_every_header_symbol():
    syms = N.header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(N.lib, s)]
    assert not missing, missing
    # and the binding declares a signature for each of them
    assert set(syms) <= set(N._SIGNATURES), set(syms) - set(N._SIGNATURES)


def test_abi_version_and_errors():
    assert N.lib.gol_abi_version() == 2  # round 5: the canonical state hash
    for code in range(7):
        assert N.lib.gol_strerror(code)
    assert N.lib.gol_strerror(99) == b"unknown error"


def test_config_struct_layout_matches_header(tmp_path):
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "gol.h"\n'
                   'int main(void){printf("%zu %zu %zu %zu\\n", sizeof(gol_config),'
                   ' offsetof(gol_config, topology), offsetof(gol_config, device),'
                   ' offsetof(gol_config, vis_height)); return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    assert got == [ctypes.sizeof(N.GolConfig), N.GolConfig.topology.offset,
                   N.GolConfig.device.offset, N.GolConfig.vis_height.offset]


@pytest.mark.parametrize("H,n", [(262144, 8), (262144, 3), (10, 10), (11, 4), (4096, 1), (7, 2)])
def test_shard_rows_partition(H, n):
    prev_end = 0
    sizes = []
    for r in range(n):
        r0, rows = N.shard_rows(H, r, n)
        assert (r0, rows) == shard_rows_py(H, r, n)
        assert r0 == prev_end
        prev_end = r0 + rows
        sizes.append(rows)
    assert prev_end == H and max(sizes) - min(sizes) <= 1


def test_shard_rows_rejects_bad_args():
    for args in [(0, 0, 1), (10, 2, 2), (10, -1, 2), (1, 0, 2)]:
        with pytest.raises(N.GolError) as ei:
            N.shard_rows(*args)
        assert ei.value.code == N.GOL_EINVAL


def test_no_cpu_fallback():
    if N.device_count() > 0:
        pytest.skip("a HIP device is present")
    from gameoflife.engine import GolEngine
    with pytest.raises(N.GolError) as ei:
        GolEngine(64, 64)
    assert ei.value.code == N.GOL_ENODEV
    assert b"no CPU fallback" in N.lib.gol_last_error(None)


def test_native_frontend_links_c_abi_only():
    exe = os.path.join(ROOT, "akka-game-of-life_amd", "bin", "gol_frontend")
    assert os.path.exists(exe)
    # built with g++ against include/gol.h: no HIP runtime symbols referenced directly
    syms = subprocess.run(["nm", "-D", "--undefined-only", exe], capture_output=True, text=True).stdout
    assert "gol_create" in syms and "hipMalloc" not in syms
    if N.device_count() == 0:
        p = subprocess.run([exe, "generations=1", "log.file=-"], capture_output=True, text=True)
        assert p.returncode == 1 and "no HIP device" in p.stderr


def test_create_validates_geometry():
    from gameoflife.engine import GolEngine
    for kw in [dict(width=33, height=8),                       # torus needs width % 32 == 0
               dict(width=64, height=8, rule=__import__("gameoflife").Rule(0x200, 0)),
               dict(width=64, height=8, row0=5, rows=4)]:
        with pytest.raises(N.GolError) as ei:
            GolEngine(**kw)
        assert ei.value.code == N.GOL_EINVAL, kw


def test_codec_matches_oracle_layout():
    rng = np.random.default_rng(1)
    for W, H in [(1, 1), (7, 7), (32, 3), (33, 5), (100, 9), (4096, 2)]:
        c = (rng.random((H, W)) < 0.5).astype(np.uint8)
        p = codec.pack(c)
        assert p.dtype == np.uint32 and p.shape == (H, (W + 31) // 32)
        assert (p == O.pack(c)).all()
        assert (codec.unpack(p, W) == c).all()


def test_layout_rule_is_geometry_only(monkeypatch):
    # libgol's own rule (gol_device_layout) and its Python restatement agree,
    # and no environment variable moves it (round 4's GOL_LAYOUT is gone)
    from gameoflife import _native as N
    for env in (None, "quads", "pairs"):
        if env is None:
            monkeypatch.delenv("GOL_LAYOUT", raising=False)
        else:
            monkeypatch.setenv("GOL_LAYOUT", env)
        for w in (32, 64, 96, 128, 320, 352, 992, 1024, 4096, 65536, 262144):
            for topo in (N.GOL_TORUS, N.GOL_REF_CLIPPED):
                assert N.device_layout(w, topo) == N.device_ilv(w, topo)
        assert [N.device_layout(w) for w in (32, 64, 96, 128, 192, 256)] == [1, 2, 1, 2, 2, 2]
        assert N.device_layout(128, N.GOL_REF_CLIPPED) == 1


def test_new_struct_layouts_match_header(tmp_path):
    """gol_profile_stats and gol_runtime_info: ctypes mirrors match the C
    layout (a JNI / Panama binding would read the same offsets)."""
    src = tmp_path / "sz2.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "gol.h"\n'
                   'int main(void){printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(gol_profile_stats),'
                   ' offsetof(gol_profile_stats, exchange_ms), offsetof(gol_profile_stats, pass_tail_ms),'
                   ' sizeof(gol_runtime_info), offsetof(gol_runtime_info, rccl_library),'
                   ' offsetof(gol_runtime_info, gol_library)); return 0;}\n')
    exe = tmp_path / "sz2"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    assert got == [ctypes.sizeof(N.GolProfileStats), N.GolProfileStats.exchange_ms.offset,
                   N.GolProfileStats.pass_tail_ms.offset, ctypes.sizeof(N.GolRuntimeInfo),
                   N.GolRuntimeInfo.rccl_library.offset, N.GolRuntimeInfo.gol_library.offset]


def test_runtime_info_names_the_rocm_stack():
    """gol_runtime_info_get is host-only: the HIP runtime and RCCL libgol is
    bound to, and where they were loaded from.  In a process that loaded
    libgol before torch (bench.py imports no torch; tests/conftest.py loads
    libgol first) that is /opt/rocm's stack."""
    info = N.runtime_info()
    assert info["hip_library"].startswith("/opt/rocm") and "libamdhip64" in info["hip_library"]
    assert info["rccl_library"].startswith("/opt/rocm") and "librccl" in info["rccl_library"]
    assert info["gol_library"].endswith("libgol.so")
    assert info["rccl_version"] >= 22000 and info["rccl"].count(".") == 2
    assert info["hip_runtime_version"] > 0


def test_bench_imports_no_torch():
    """bench.py runs without torch: importing it and
    building its argument parser leaves torch unloaded."""
    code = ("import sys; sys.argv=['bench.py']; import bench; bench.parse(); "
            "print('torch' in sys.modules)")
    out = subprocess.run([os.sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, check=True)
    assert out.stdout.strip() == "False"
