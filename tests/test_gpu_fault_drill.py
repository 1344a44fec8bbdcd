"""GPU: the multi-GPU bench's fault drill (BASELINE.json configs[4];
gameoflife.elastic.ring_fault_drill, bench.py fault_drill) with its ranks as
loopback-ring contexts on one GPU -- one host thread each, as one process per
GPU would be, running the RCCL schedule's exact halo operations.

A rank drops its communicator and context after generation 25 of 50; the rank
above it restores the lost block's last checkpoint file, replays it alone
from the light cone in its neighbours' files (gol_replay) and merges it with
its own rows; the survivors rebuild the ring (gol_comm_abort + a new loopback
ring, ranks renumbered) and step on.  Every global hash the drill reports and
the final board equal the oracle's (small boards) or the golden table
(65536^2, tests/golden/bench_65536.json).  Mirrors BoardCreator.scala:120-154
and CellActor.scala:34,71-74,86."""
import json
import os
import threading
import uuid

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _drill(W, H, world, seed, ckpt_dir, victim=3, kill_at=25, gens=50, every=10):
    from gameoflife import _native as N
    from gameoflife.elastic import ring_fault_drill
    from gameoflife.engine import GolEngine
    prefix = uuid.uuid4().hex
    make = lambda r0, n: GolEngine(W, H, topology="torus", rule="life", row0=r0, rows=n)  # noqa: E731
    join = lambda e, tag, r, w: e.comm_init_loopback(f"{prefix}_{tag}", r, w)  # noqa: E731
    engs = []
    for r in range(world):
        row0, rows = N.shard_rows(H, r, world)
        e = make(row0, rows)
        e.comm_init_loopback(f"{prefix}_first", r, world)
        engs.append(e)
    out, errs = [None] * world, []

    def work(r):
        try:
            out[r] = ring_fault_drill(engs[r], make, join, r, world, W, H, ckpt_dir, seed=seed, victim=victim,
                                      kill_at=kill_at, gens=gens, every=every)
        except Exception as exc:  # noqa: BLE001 -- reported to the test thread
            errs.append(exc)

    ts = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(300)
    try:
        assert not any(t.is_alive() for t in ts), "a rank hung"
        if errs:
            raise errs[0]
        finals = [(rep["rows_after"], e.snapshot()) for e, rep in out if e is not None]
        return out, finals
    finally:
        for e, _ in (o for o in out if o is not None):
            if e is not None:
                e.close()


def _check(out, want, world, victim, gens=50, kill_at=25):
    """Every survivor's report against the expected global hashes `want`
    (want[k] = epoch k + 1)."""
    lost = [r for r, (e, rep) in enumerate(out) if e is None]
    assert lost == [min(victim, world - 1)]
    for e, rep in out:
        if e is None:
            continue
        assert rep["world_after"] == world - 1
        c = rep["checkpoint_epoch"]
        assert c == 20 and rep["replayed_generations"] == kill_at - c
        assert rep["before"] == want[:kill_at]
        assert rep["replayed"] == want[c:kill_at]
        assert rep["at_recovery"] == want[kill_at - 1]
        assert rep["after"] == want[kill_at:gens]
        assert rep["final"] == want[gens - 1]


@pytest.mark.parametrize("world,victim", [(4, 3), (3, 3), (2, 3), (4, 0)])
def test_fault_drill_loopback_matches_oracle(gpu, tmp_path, world, victim):
    W, H, seed = 32 * 200, 96, 0x5EED + world
    board = O.seed_packed(W, H, seed)
    final_cpu, want = O.run_packed(board, W, 50, O.TORUS, O.LIFE)
    out, finals = _drill(W, H, world, seed, str(tmp_path), victim=victim)
    want = [int(x) for x in want]
    _check(out, want, world, victim)
    # the survivors' final rows, in row order, are the oracle's board at 50
    row = 0
    for (row0, rows), snap in sorted(finals, key=lambda x: x[0][0]):
        assert row0 == row
        np.testing.assert_array_equal(snap, final_cpu[row0:row0 + rows])
        row += rows
    assert row == H


def test_fault_drill_loopback_65536_golden(gpu, tmp_path):
    """At a size where a shard is many bands and a checkpoint file 128 MiB:
    four ranks of 65536^2, rank 3 lost; every hash against the golden table."""
    S = 65536
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bench_65536.json")) as f:
        golden = [int(x, 16) for x in json.load(f)["hashes"]]
    out, _ = _drill(S, S, 4, 0x5EED, str(tmp_path))
    _check(out, golden[1:51], 4, 3)


def test_fault_drill_loopback_262144_golden(gpu, tmp_path):
    """The bench's own N = 8 drill (configs[4] on configs[3]'s board): eight
    ranks of 262144^2 (1 GiB shards), rank 3 lost after 25 of 50, every hash
    against bench_262144.json.  The checkpoint files peak at two epochs of the
    board (16 GiB); without that much room in the test's directory it skips."""
    import shutil
    S = 262144
    if shutil.disk_usage(str(tmp_path)).free < 2 * S * S // 8 + (4 << 30):
        pytest.skip("no room for two epochs of 262144^2 checkpoint files")
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bench_262144.json")) as f:
        golden = [int(x, 16) for x in json.load(f)["hashes"]]
    out, _ = _drill(S, S, 8, 0x5EED, str(tmp_path))
    _check(out, golden[1:51], 8, 3)
    print("drill wall per survivor: recovery %.3f s, after %.3f s, checkpoints %.3f s" % max(
        (rep["recovery_s"], rep["after_s"], rep["checkpoint_s"]) for e, rep in out if e is not None))
