import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "akka-game-of-life_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: longer CPU test")


def _ensure_built():
    """Build the oracle and libgol in-tree if they are missing (hipcc
    cross-compiles gfx950 without a GPU)."""
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                       stdout=subprocess.DEVNULL)
    if not os.path.exists(os.path.join(PKG, "lib", "libgol.so")) and shutil.which("hipcc"):
        subprocess.run(["make", "-C", PKG, "-j4"], check=True, stdout=subprocess.DEVNULL)


_ensure_built()

# Load libgol before any test module can import torch: the dynamic linker
# then binds libgol -- and anything loaded later that asks for the same
# sonames -- to /opt/rocm's HIP runtime and RCCL, the stack bench.py (which
# imports no torch) and a JVM host run on.  The terminal summary names it.
try:
    from gameoflife import _native as _gol_native  # noqa: F401
except ImportError:
    _gol_native = None


def _gpu_available() -> bool:
    try:
        from gameoflife import _native as N
        return N.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not _gpu_available():
        pytest.fail("no HIP device: -m gpu tests need an MI355X")
    return 0


def pytest_terminal_summary(terminalreporter):
    """The HIP runtime and RCCL libgol ran on (gol_runtime_info_get) and, on
    GPU runs, how many HIP statuses RCCL calls left behind during the session
    (libgol absorbs and counts them)."""
    mod = sys.modules.get("gameoflife._native")
    if mod is None:
        return
    info = mod.runtime_info()
    terminalreporter.write_line(
        f"libgol runtime: HIP {info['hip_runtime']} ({info['hip_library']}), RCCL {info['rccl']} "
        f"({info['rccl_library']}), torch loaded in this session: {info['torch_loaded']}")
    if not _gpu_available():
        return
    n, last = mod.absorbed()
    terminalreporter.write_line(f"libgol: HIP statuses absorbed after RCCL calls this session: {n}"
                                + (f" (last: {last})" if n else ""))

