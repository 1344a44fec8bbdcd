"""Probe of the HIP runtime's pending-status semantics on this image (which
calls leave, keep or clear the thread's hipGetLastError status); used to
shape the HIP status discipline."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))
from gameoflife import _native as N  # noqa: E402
from gameoflife.engine import GolEngine  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
for f in ("hipSetDevice", "hipGetLastError", "hipPeekAtLastError", "hipDeviceSynchronize"):
    getattr(hip, f).restype = ctypes.c_int
hip.hipSetDevice.argtypes = [ctypes.c_int]
hip.hipGetDevice.argtypes = [ctypes.POINTER(ctypes.c_int)]


def fresh_error():
    hip.hipGetLastError()
    return hip.hipSetDevice(9999)


d = ctypes.c_int()
print("failing hipSetDevice returns", fresh_error(), "peek", hip.hipPeekAtLastError(), "get", hip.hipGetLastError(),
      "get again", hip.hipGetLastError())
fresh_error(); hip.hipGetDevice(ctypes.byref(d))
print("after a successful hipGetDevice: get", hip.hipGetLastError())
fresh_error(); hip.hipSetDevice(0)
print("after a successful hipSetDevice: get", hip.hipGetLastError())
fresh_error(); hip.hipDeviceSynchronize()
print("after a successful hipDeviceSynchronize: get", hip.hipGetLastError())
with GolEngine(32 * 64, 64) as e:
    e.seed(1)
    fresh_error(); e.seed(2)
    print("after gol_seed (one hipLaunchKernel + stream sync): get", hip.hipGetLastError())
    fresh_error(); e.step(4)
    print("after gol_step (launches only): get", hip.hipGetLastError())
    fresh_error(); e.hash()
    print("after gol_hash: get", hip.hipGetLastError())
print("absorbed", N.absorbed())
