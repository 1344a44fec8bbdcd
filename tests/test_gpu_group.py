"""GPU: the sharded schedule (interior rows || halo exchange, then boundary
rows; G-deep halos) through an in-process shard group, and the fault path
(BASELINE.json config 5: kill a shard mid-run, re-spawn it from the last
checkpoint, hashes unchanged).  Bit-exact against the CPU oracle."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def make_group(W, H, n, topology="torus", rule="life", gpp=0, seed=77, cells=None):
    from gameoflife.engine import GolEngine, ShardGroup
    from gameoflife.shard import shard_rows_py
    shards = []
    full = O.pack(cells) if cells is not None else O.seed_packed(W, H, seed)
    for k in range(n):
        r0, rows = shard_rows_py(H, k, n)
        e = GolEngine(W, H, topology=topology, rule=rule, row0=r0, rows=rows)
        e.set_tuning(gens_per_pass=gpp)
        e.load(full[r0:r0 + rows])
        shards.append(e)
    return shards, ShardGroup(shards), full


@pytest.mark.parametrize("n", [2, 3, 5, 8])
@pytest.mark.parametrize("gpp", [1, 2, 6, 12])
def test_group_torus_matches_oracle(gpu, n, gpp):
    W, H, gens = 32 * 300, 83, 13  # uneven shards (83 rows over n), rows <= 2G for some
    shards, g, full = make_group(W, H, n, gpp=gpp)
    got = g.step(gens, hashes=True)
    board = g.snapshot()
    ref, want = O.run_packed(full, W, gens, O.TORUS, O.LIFE)
    np.testing.assert_array_equal(got, want)
    assert (board == ref).all()
    g.close()
    for s in shards:
        s.close()


@pytest.mark.parametrize("n", [2, 5])
def test_group_whole_row_waves(gpu, n):
    """A 4096-column torus (one wave of pairs per row): the group's
    10-generation passes run whole-row waves in every shard's interior and
    boundary launches."""
    W, H, gens = 4096, 403, 40
    shards, g, full = make_group(W, H, n, gpp=10, seed=n)
    got = g.step(gens, hashes=True)
    board = g.snapshot()
    ref, want = O.run_packed(full, W, gens, O.TORUS, O.LIFE)
    np.testing.assert_array_equal(got, want)
    assert (board == ref).all()
    g.close()
    for s in shards:
        s.close()


@pytest.mark.parametrize("n", [2, 4])
@pytest.mark.parametrize("gpp", [1, 3, 6])
def test_group_clipped_matches_oracle(gpu, n, gpp):
    W, H, gens = 1000, 61, 9
    rng = np.random.default_rng(n * 10 + gpp)
    cells = (rng.random((H, W)) < 0.5).astype(np.uint8)
    shards, g, full = make_group(W, H, n, topology="ref-clipped", rule="B36/S23", gpp=gpp, cells=cells)
    got = g.step(gens, hashes=True)
    board = g.snapshot()
    ref, want = O.run_packed(full, W, gens, O.REF_CLIPPED, (0x48, 0x0C))
    np.testing.assert_array_equal(got, want)
    assert (board == ref).all()
    g.close()
    for s in shards:
        s.close()


def test_group_rejects_bad_layout_and_lost_shard(gpu):
    from gameoflife import _native as N
    from gameoflife.engine import GolEngine, ShardGroup
    a = GolEngine(256, 40, row0=0, rows=20)
    b = GolEngine(256, 40, row0=21, rows=19)  # gap at row 20
    with pytest.raises(N.GolError):
        ShardGroup([a, b])
    b.close()
    b = GolEngine(256, 40, row0=20, rows=20)
    g = ShardGroup([a, b])
    g.step(3)
    b.close()  # the shard dies: the group has a hole
    with pytest.raises(N.GolError) as ei:
        g.step(1)
    assert ei.value.code == N.GOL_ESTATE and "destroyed" in ei.value.message
    g.close()
    a.close()


@pytest.mark.parametrize("ckpt_dir,mode", [(False, "light-cone"), (True, "light-cone"), (False, "rollback")])
def test_fault_kill_and_respawn_hashes_match(gpu, tmp_path, ckpt_dir, mode):
    """BASELINE.json config 5 in miniature: 8 shards, checkpoint every 10,
    shard 3 killed at generation 25 of 50 and re-spawned next to a survivor --
    alone from its checkpoint and its neighbours' light cone (the others keep
    their state), or by a global rollback: every per-generation hash equals
    the uninterrupted run's, and the final board equals the oracle's."""
    from gameoflife import _native as N
    from gameoflife.fault import ShardedSimulation
    W, H = 32 * 256, 1024
    devices = list(range(N.device_count()))
    ref = ShardedSimulation(W, H, 8, devices, checkpoint_every=10)
    want = ref.step(50)
    ref_board = ref.snapshot()
    ref.close()

    sim = ShardedSimulation(W, H, 8, devices, checkpoint_every=10,
                            checkpoint_dir=str(tmp_path) if ckpt_dir else None)
    got = sim.step(25)
    # the checkpoint of epoch 20 has landed (explicit: whether an in-flight
    # copy has reached host memory is timing on a live in-process shard)
    sim.kill(3, checkpoint_landed=True)
    with pytest.raises(RuntimeError):
        sim.step(1)
    replayed = sim.respawn(3, mode=mode)
    assert len(replayed) == 5 and sim.epoch == 25
    if mode == "light-cone":  # shard 3's own partial hashes of generations 21..25
        row0, rows = N.shard_rows(H, 3, 8)
        b = O.seed_packed(W, H, 0x5EED)
        b, _ = O.run_packed(b, W, 20, want_hashes=False)
        for g in range(5):
            b, _ = O.run_packed(b, W, 1, want_hashes=False)
            assert replayed[g] == O.hash_packed(b[row0:row0 + rows], W, row0=row0), g
    got += sim.step(25)
    assert got == want
    assert sim.hashes == want
    assert (sim.snapshot() == ref_board).all()
    assert any(e.startswith("respawn shard 3") for e in sim.events)
    sim.close()

    board0 = O.seed_packed(W, H, 0x5EED)
    final, oh = O.run_packed(board0, W, 50, O.TORUS, O.LIFE)
    assert [int(x) for x in oh] == want
    assert (final == ref_board).all()


@pytest.mark.parametrize("topology", ["torus", "ref-clipped"])
def test_recurring_crashes_light_cone(gpu, topology):
    """Crashes on the reference's schedule (errors.delay / errors.every /
    max-crashes, board.crash_schedule): each lost shard is re-spawned alone
    from its checkpoint and its neighbours' light cone -- including light
    cones deeper than a neighbour shard (checkpoint every 12, shards of 9-10
    rows) -- and the hashes equal the uninterrupted oracle run."""
    from gameoflife import _native as N
    from gameoflife.board import SimulationParams, crash_schedule
    from gameoflife.fault import ShardedSimulation
    W, H, gens = 32 * 100 + (0 if topology == "torus" else 13), 77, 60
    p = SimulationParams(start_delay_ms=0, tick_ms=100, first_error_after_ms=500, error_every_ms=1100,
                         max_number_of_crashes=5)
    crashes = crash_schedule(p, gens, seed=11)
    assert len(crashes) == 5
    sim = ShardedSimulation(W, H, 8, list(range(N.device_count())), topology=topology, checkpoint_every=12)
    got = sim.run(gens, crashes)
    board = sim.snapshot()
    assert sum(e.startswith("respawn") for e in sim.events) == 5
    sim.close()
    topo = O.TORUS if topology == "torus" else O.REF_CLIPPED
    final, want = O.run_packed(O.seed_packed(W, H, 0x5EED), W, gens, topo, O.LIFE)
    assert got == [int(x) for x in want]
    assert (board == final).all()


def test_recurring_crashes_async_checkpoints(gpu):
    """The same recurring-crash schedule with the checkpoints taken in the
    background (gol_checkpoint_async, two page-locked buffer sets): each loss
    recovers from the last checkpoint that has landed, and every hash equals
    the uninterrupted oracle run."""
    from gameoflife import _native as N
    from gameoflife.board import SimulationParams, crash_schedule
    from gameoflife.fault import ShardedSimulation
    W, H, gens = 32 * 100, 77, 60
    p = SimulationParams(start_delay_ms=0, tick_ms=100, first_error_after_ms=500, error_every_ms=1100,
                         max_number_of_crashes=5)
    crashes = crash_schedule(p, gens, seed=11)
    sim = ShardedSimulation(W, H, 8, list(range(N.device_count())), checkpoint_every=12, async_checkpoints=True)
    got = sim.run(gens, crashes)
    board = sim.snapshot()
    assert sum(e.startswith("respawn") for e in sim.events) == 5
    assert sum(e.startswith("checkpoint@") for e in sim.events) >= 5
    sim.close()
    final, want = O.run_packed(O.seed_packed(W, H, 0x5EED), W, gens, O.TORUS, O.LIFE)
    assert got == [int(x) for x in want]
    assert (board == final).all()


@pytest.mark.parametrize("landed", [False, True])
def test_kill_while_async_checkpoint_in_flight(gpu, landed):
    """a shard lost while its background checkpoint is in flight.
    If its part had not landed, the whole set is dropped and recovery replays
    from the previous committed checkpoint (a longer light cone); if it had,
    the set is the recovery point.  Either way every hash equals the oracle's,
    and the replayed partials complete the recorded global hashes."""
    from gameoflife import _native as N
    from gameoflife.fault import ShardedSimulation
    W, H, gens = 32 * 100, 80, 40
    sim = ShardedSimulation(W, H, 8, list(range(N.device_count())), checkpoint_every=10, async_checkpoints=True)
    got = sim.step(20)              # the epoch-20 checkpoint is now in flight
    sim.kill(3, checkpoint_landed=landed)
    replayed = sim.respawn(3)
    c = 20 if landed else 10
    assert f"respawn shard 3 on device {sim.placement[3]}, light cone {c}->20" in sim.events
    assert len(replayed) == 20 - c
    assert any("dropped" in e for e in sim.events) != landed
    got += sim.step(gens - 20)
    board = sim.snapshot()
    sim.close()
    final, want = O.run_packed(O.seed_packed(W, H, 0x5EED), W, gens, O.TORUS, O.LIFE)
    assert got == [int(x) for x in want]
    assert (board == final).all()


def test_snapshot_query_reports_landing(gpu):
    from gameoflife import _native as N
    from gameoflife.engine import GolEngine
    with GolEngine(32 * 64, 64) as e:
        e.seed(5)
        with pytest.raises(N.GolError):
            e.snapshot_landed()  # nothing in flight
        buf = e.host_buffer()
        e.snapshot_async(buf)
        e.sync()
        import time
        t0 = time.time()
        while not e.snapshot_landed() and time.time() - t0 < 10:
            time.sleep(0.001)
        assert e.snapshot_landed()
        assert e.snapshot_wait() == 0
        assert (buf == O.seed_packed(32 * 64, 64, 5)).all()

