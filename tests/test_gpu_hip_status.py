"""GPU: the HIP status discipline around RCCL setup and teardown (DESIGN.md
section 2, "HIP status discipline").

Round 2 cleared any pending HIP status before every launch because a status
left behind after an RCCL teardown had failed a later seed launch.  Now
kernels are launched with hipLaunchKernel (its return value is the launch's
own status), every status libgol reports or logs is taken off the thread, and
what RCCL's own HIP calls leave behind is absorbed right after each RCCL call
(gol_diag_absorbed counts it).  These tests check, after every entry point,
that the thread holds no pending HIP status, on the path config 5 takes when
a backend leaves the ring (BoardCreator.scala:129-130,138-154): comm_init ->
step -> comm_abort -> comm_init -> step, bit-exact against the oracle."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

W, H, G = 32 * 300, 96, 14


def _clean(what):
    from gameoflife import _native as N
    code = N.take_hip_error()
    assert code == 0, f"HIP status {code} pending after {what}"


def test_self_ring_abort_rejoin_bit_exact(gpu):
    from gameoflife import _native as N
    from gameoflife.engine import GolEngine
    N.take_hip_error()  # start from a clean thread, whatever ran before
    board = O.seed_packed(W, H, 7)
    _, want = O.run_packed(board, W, 2 * G, O.TORUS, O.LIFE)
    final_cpu, _ = O.run_packed(board, W, 2 * G, O.TORUS, O.LIFE, want_hashes=False)
    n0, _ = N.absorbed()
    e = GolEngine(W, H)
    _clean("gol_create")
    e.load(board)
    _clean("gol_load")
    e.comm_init(N.unique_id(), 0, 1)
    _clean("gol_comm_init")
    h1 = e.step(G, hashes=True)
    _clean("gol_step (self-ring)")
    e.comm_abort()
    _clean("gol_comm_abort")
    e.comm_init(N.unique_id(), 0, 1)
    _clean("gol_comm_init after abort")
    h2 = e.step(G, hashes=True)
    _clean("gol_step after the ring was rebuilt")
    np.testing.assert_array_equal(np.concatenate([h1, h2]), want)
    assert np.array_equal(e.snapshot(), final_cpu)
    _clean("gol_snapshot")
    e.close()
    _clean("gol_destroy of a context with a communicator")
    n1, last = N.absorbed()
    print(f"RCCL statuses absorbed: {n1 - n0} ({last or 'none'})")


def test_fresh_context_after_ring_teardown(gpu):
    """Destroy a ring context, then create and seed a fresh one: the seed
    launch must not inherit anything from the teardown (the round-2 failure)."""
    from gameoflife import _native as N
    from gameoflife.engine import GolEngine
    N.take_hip_error()
    with GolEngine(W, H) as e:
        e.seed(3)
        e.comm_init(N.unique_id(), 0, 1)
        e.step(G)
        e.sync()
    _clean("gol_destroy of a ring context")
    with GolEngine(W, H) as e2:
        _clean("gol_create after the teardown")
        e2.seed(0x5EED)
        _clean("gol_seed after the teardown")
        got = e2.step(G, hashes=True)
        _clean("gol_step after the teardown")
    _, want = O.run_packed(O.seed_packed(W, H, 0x5EED), W, G, O.TORUS, O.LIFE)
    np.testing.assert_array_equal(got, want)


def test_callers_pending_status_is_not_pinned_on_a_launch(gpu):
    """A HIP status the caller left pending (here: a failed hipSetDevice made
    directly through the runtime) must not fail libgol's launches: they report
    their own status (hipLaunchKernel), not the thread's pending one.  (Whether
    it is still pending afterwards is the runtime's business: some successful
    runtime calls on the hashed path reset it, scripts/hip_status_probe.py.)"""
    from gameoflife import _native as N
    from gameoflife.engine import GolEngine
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipSetDevice.restype = ctypes.c_int
    hip.hipSetDevice.argtypes = [ctypes.c_int]
    with GolEngine(W, H) as e:
        e.seed(11)
        N.take_hip_error()
        assert hip.hipSetDevice(9999) != 0  # invalid device: pending on this thread
        got = e.step(G, hashes=True)  # launches through hipLaunchKernel
        assert hip.hipSetDevice(9999) != 0
        e.step(G)  # the unhashed path: launches only
        e.sync()
        got2 = e.hash()
        N.take_hip_error()
    _, want = O.run_packed(O.seed_packed(W, H, 11), W, 2 * G, O.TORUS, O.LIFE)
    np.testing.assert_array_equal(got, want[:G])
    assert got2 == int(want[-1])
