"""GPU: the per-rank diagnostics bench.py reports at N > 1 and the loopback
ring's failure paths.

* gol_profile_stats_read splits a sharded pass into its interior launch, the
  halo exchange on the comm stream (HIP events around the RCCL group) and the
  boundary launches, with the halo bytes posted -- checked on a 1-rank RCCL
  self-ring (ncclSend / ncclRecv to itself) and on loopback rings;
* the loopback ring (the in-process stand-in for RCCL that runs libgol's exact
  halo operation list) must fail fast and cleanly when a rank never posts its
  operations: the waiting rank times out with GOL_ECOMM, withdraws its queued
  operations (they hold its plane pointers), and every other rank of that ring
  gets GOL_ECOMM at once; boards stay at their last complete epoch and a new
  ring continues bit-exact."""
import threading
import time
import uuid

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _engine(W, H, **kw):
    from gameoflife.engine import GolEngine
    return GolEngine(W, H, topology="torus", rule="life", **kw)


def test_profile_stats_self_ring(gpu):
    from gameoflife import _native as N
    W, H, G = 32 * 256, 96, 4
    with _engine(W, H) as e:
        e.seed(11)
        e.comm_init(N.unique_id(), 0, 1)
        e.set_tuning(gens_per_pass=G)
        e.step(G)
        e.sync()
        e.profile(True)
        e.profile_reset()
        e.step(3 * G)
        e.sync()
        st = e.profile_stats()
        pitch_bytes = 256 * 4  # 256 words per row, already a multiple of 64
        assert st["launches"] == 3 and st["generations"] == 3 * G
        assert st["exchanges"] == 3 and st["boundary_launches"] == 3
        assert st["halo_bytes_sent"] == 3 * 2 * G * pitch_bytes == st["halo_bytes_received"]
        assert st["kernel_ms"] > 0 and st["exchange_ms"] > 0 and st["boundary_ms"] > 0
        # the exposed exchange and the boundary tail end after the interior
        # launch by at most the whole exchange / boundary window
        assert 0 <= st["exchange_exposed_ms"] <= st["exchange_ms"] + 1e-3
        assert 0 <= st["pass_tail_ms"] and st["pass_tail_ms"] >= st["exchange_exposed_ms"] - 1e-3
        ms, n, g = e.profile_read()
        assert (ms, n, g) == (st["kernel_ms"], st["launches"], st["generations"])
        e.profile_reset()
        st = e.profile_stats()
        assert st["exchanges"] == 0 and st["halo_bytes_sent"] == 0 and st["kernel_ms"] == 0
        e.profile(False)
        e.step(G)
        e.sync()
        st = e.profile_stats()
        assert st["exchanges"] == 0 and st["halo_bytes_sent"] == 2 * G * pitch_bytes  # counted unprofiled too


def test_profile_stats_unsharded_has_no_exchange(gpu):
    with _engine(32 * 128, 64) as e:
        e.seed(3)
        e.set_tuning(gens_per_pass=6)
        e.profile(True)
        e.profile_reset()
        e.step(12)
        st = e.profile_stats()
        assert st["launches"] == 2 and st["exchanges"] == 0 and st["boundary_launches"] == 0
        assert st["halo_bytes_sent"] == 0 and st["clock_ghz"] >= 0


def _ring(W, H, world, board, gpp=0, key=None):
    from gameoflife import _native as N
    key = key or uuid.uuid4().hex
    engs = []
    for r in range(world):
        row0, rows = N.shard_rows(H, r, world)
        e = _engine(W, H, row0=row0, rows=rows)
        e.set_tuning(gens_per_pass=gpp)
        e.load(board[row0:row0 + rows])
        e.comm_init_loopback(key, r, world)
        engs.append(e)
    return engs


def _threads(engs, fn):
    out, errs = [None] * len(engs), []

    def work(r):
        try:
            out[r] = fn(r, engs[r])
        except Exception as exc:  # noqa: BLE001 -- handed to the test thread
            errs.append(exc)

    ts = [threading.Thread(target=work, args=(r,)) for r in range(len(engs))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert not any(t.is_alive() for t in ts), "a rank hung"
    if errs:
        raise errs[0]
    return out


def test_loopback_stats_per_rank(gpu):
    W, H, G = 32 * 128, 60, 3
    board = O.seed_packed(W, H, 5)
    engs = _ring(W, H, 3, board, gpp=G)
    try:
        def run(r, e):
            e.profile(True)
            e.profile_reset()
            e.step(2 * G)
            e.sync()
            return e.profile_stats()
        for st in _threads(engs, run):
            assert st["exchanges"] == 2 and st["boundary_launches"] == 2 and st["launches"] == 2
            assert st["halo_bytes_sent"] == 2 * 2 * G * 128 * 4
    finally:
        for e in engs:
            e.close()


def test_loopback_peer_that_never_posts_fails_fast(gpu, monkeypatch):
    from gameoflife import _native as N
    monkeypatch.setenv("GOL_LOOPBACK_TIMEOUT_MS", "1500")
    W, H, G = 32 * 64, 40, 4
    board = O.seed_packed(W, H, 4242)
    engs = _ring(W, H, 2, board, gpp=G)
    try:
        # rank 0 steps, rank 1 skips the step: rank 0 waits out the timeout
        t0 = time.monotonic()
        with pytest.raises(N.GolError) as ei:
            engs[0].step(G)
        assert ei.value.code == N.GOL_ECOMM and "timed out" in ei.value.message
        assert time.monotonic() - t0 < 30
        assert engs[0].epoch == 0
        # the ring has failed: rank 1's step and all-reduce return at once,
        # without matching rank 0's withdrawn operations
        t1 = time.monotonic()
        with pytest.raises(N.GolError) as ei:
            engs[1].step(G)
        assert ei.value.code == N.GOL_ECOMM and time.monotonic() - t1 < 1.0
        with pytest.raises(N.GolError) as ei:
            engs[1].allreduce_u64(np.array([1], dtype=np.uint64))
        assert ei.value.code == N.GOL_ECOMM
        assert engs[1].epoch == 0
        assert N.take_hip_error() == 0
        # both leave; a new ring continues bit-exact from epoch 0
        for e in engs:
            e.comm_abort()
        key = uuid.uuid4().hex
        for r, e in enumerate(engs):
            e.comm_init_loopback(key, r, 2)
        got = _threads(engs, lambda r, e: e.allreduce_u64(e.step(2 * G, hashes=True)))
        final = np.vstack([e.snapshot() for e in engs])
    finally:
        for e in engs:
            e.close()
    final_cpu, want = O.run_packed(board, W, 2 * G, O.TORUS, O.LIFE)
    np.testing.assert_array_equal(got[0], want)
    np.testing.assert_array_equal(final, final_cpu)


def test_loopback_rejects_duplicate_rank_and_failed_key(gpu):
    from gameoflife import _native as N
    W, H = 32 * 64, 40
    key = uuid.uuid4().hex
    a, b, c = _engine(W, H, row0=0, rows=20), _engine(W, H, row0=0, rows=20), _engine(W, H, row0=20, rows=20)
    try:
        a.comm_init_loopback(key, 0, 2)
        with pytest.raises(N.GolError) as ei:
            b.comm_init_loopback(key, 0, 2)
        assert ei.value.code == N.GOL_EINVAL
        c.comm_init_loopback(key, 1, 2)
        a.comm_abort()  # leaving with a peer still in the ring fails the ring
        with pytest.raises(N.GolError) as ei:
            c.allreduce_u64(np.array([1], dtype=np.uint64))
        assert ei.value.code == N.GOL_ECOMM
        with pytest.raises(N.GolError) as ei:
            b.comm_init_loopback(key, 0, 2)
        assert ei.value.code == N.GOL_ESTATE
    finally:
        for e in (a, b, c):
            e.close()


def test_loopback_allreduce_count_mismatch_fails_both(gpu, monkeypatch):
    from gameoflife import _native as N
    monkeypatch.setenv("GOL_LOOPBACK_TIMEOUT_MS", "20000")
    W, H = 32 * 64, 40
    board = O.seed_packed(W, H, 1)
    engs = _ring(W, H, 2, board)
    try:
        codes = [None, None]

        def run(r, e):
            time.sleep(0.2 * r)
            try:
                e.allreduce_u64(np.zeros(2 + r, dtype=np.uint64))
            except N.GolError as exc:
                codes[r] = exc.code
        t0 = time.monotonic()
        _threads(engs, run)
        assert time.monotonic() - t0 < 10  # the first rank is woken, not left to time out
        assert sorted(codes) == sorted([N.GOL_ECOMM, N.GOL_EINVAL])
    finally:
        for e in engs:
            e.close()


def test_runtime_info_on_the_gpu_box(gpu):
    """The pytest GPU session runs libgol on /opt/rocm's HIP runtime and RCCL
    (tests/conftest.py loads libgol before any torch import), the stack
    bench.py reports in its "runtime" field."""
    from gameoflife import _native as N
    info = N.runtime_info()
    assert info["hip_library"].startswith("/opt/rocm") and info["rccl_library"].startswith("/opt/rocm")
    assert info["hip_runtime_version"] > 0 and info["hip_driver_version"] > 0
