"""Asynchronous snapshots (gol_snapshot_async / gol_snapshot_wait): the board
at the snapshot epoch reaches the host while later generations run, for the
pair layout (de-interleaved on the device) and the row-major layouts, as a
stand-alone context, a 1-rank RCCL self-ring and shards of a group; plus the
state errors.  Replaces LoggerActor's periodic board dump
(LoggerActor.scala:30-46) fed by CellStateMsg (CellActor.scala:89).  Bar:
bit-exact against the CPU oracle at the snapshot epoch."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _want(board, W, gens, topo=O.TORUS, rule=O.LIFE):
    return O.run_packed(board, W, gens, topo, rule, want_hashes=False)[0]


@pytest.mark.parametrize("W,H,topology", [(32 * 512, 300, "torus"),     # pair layout
                                          (32 * 100, 50, "torus"),      # pair layout, pitch 128 != 100 words
                                          (32 * 301, 77, "torus"),      # odd words: row-major torus
                                          (32 * 40 + 13, 61, "ref-clipped")])
def test_async_snapshot_overlaps_later_steps(gpu, W, H, topology):
    from gameoflife.engine import GolEngine
    topo = O.TORUS if topology == "torus" else O.REF_CLIPPED
    board = O.seed_packed(W, H, 0x5EED) if topology == "torus" else O.pack(
        (np.random.default_rng(3).random((H, W)) < 0.4).astype(np.uint8))
    with GolEngine(W, H, topology=topology) as e:
        e.load(board)
        e.step(5)
        buf = e.host_buffer()  # page-locked
        e.snapshot_async(buf)
        got_hashes = e.step(19, hashes=True)  # queued behind the device copy, overlapping the transfer
        assert e.snapshot_wait() == 5
        np.testing.assert_array_equal(buf, _want(board, W, 5, topo))
        np.testing.assert_array_equal(e.snapshot(), _want(board, W, 24, topo))
        _, want_h = O.run_packed(_want(board, W, 5, topo), W, 19, topo, O.LIFE)
        np.testing.assert_array_equal(got_hashes, want_h)
        # a pageable buffer works too, and the buffer can be reused
        page = np.zeros_like(buf)
        e.snapshot_async(page)
        e.step(7)
        assert e.snapshot_wait() == 24
        np.testing.assert_array_equal(page, _want(board, W, 24, topo))
        e.snapshot_async(buf)
        assert e.snapshot_wait() == 31
        np.testing.assert_array_equal(buf, _want(board, W, 31, topo))


def test_async_snapshot_state_errors(gpu):
    from gameoflife import _native as N
    from gameoflife.engine import GolEngine
    with GolEngine(32 * 64, 40) as e:
        e.seed(7)
        with pytest.raises(N.GolError) as ex:
            e.snapshot_wait()
        assert ex.value.code == N.GOL_ESTATE
        buf = e.host_buffer()
        e.snapshot_async(buf)
        with pytest.raises(N.GolError) as ex:
            e.snapshot_async(buf)
        assert ex.value.code == N.GOL_ESTATE
        assert e.snapshot_wait() == 0
        np.testing.assert_array_equal(buf, O.seed_packed(32 * 64, 40, 7))
        with pytest.raises(ValueError):
            e.snapshot_async(np.zeros((40, 63), dtype=np.uint32))
    # destroying a context with a snapshot in flight waits for it
    with GolEngine(32 * 64, 40) as e:
        e.seed(9)
        keep = e.host_buffer()
        e.snapshot_async(keep)
    np.testing.assert_array_equal(keep, O.seed_packed(32 * 64, 40, 9))


def test_async_snapshot_self_ring_and_group(gpu):
    """The sharded schedules: a 1-rank RCCL self-ring (boundary rows on the
    edge stream) and the shards of an in-process group."""
    from gameoflife import _native as N
    from gameoflife.engine import GolEngine, ShardGroup
    W, H = 32 * 256, 96
    board = O.seed_packed(W, H, 0x5EED)
    with GolEngine(W, H) as e:
        e.comm_init(N.unique_id(), 0, 1)
        e.load(board)
        e.step(12)
        buf = e.host_buffer()
        e.snapshot_async(buf)
        e.step(20)
        assert e.snapshot_wait() == 12
        np.testing.assert_array_equal(buf, _want(board, W, 12))
    shards = [GolEngine(W, H, row0=r0, rows=n) for r0, n in (N.shard_rows(H, k, 3) for k in range(3))]
    for s in shards:
        s.seed(0x5EED)
    with ShardGroup(shards) as g:
        g.step(9)
        bufs = [s.host_buffer() for s in shards]
        for s, b in zip(shards, bufs):
            s.snapshot_async(b)
        g.step(6)
        assert [s.snapshot_wait() for s in shards] == [9, 9, 9]
        np.testing.assert_array_equal(np.vstack(bufs), _want(board, W, 9))
        np.testing.assert_array_equal(g.snapshot(), _want(board, W, 15))
    for s in shards:
        s.close()
