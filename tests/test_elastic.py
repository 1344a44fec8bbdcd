"""Cross-process fault path (gameoflife.elastic, BASELINE.json config 5):
checkpoint files, re-sharded restore, and the supervisor killing a backend
process mid-run and re-deploying the board on the survivors.  The CPU tests
run real backend processes with the oracle/gloo shard double
(tests/elastic_oracle_shard.py); the GPU test runs libgol backends."""
import os

import pytest

from gameoflife import elastic as E
from oracle import oracle as O

TESTS = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(TESTS)


def _env():
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([TESTS, ROOT] + [p for p in env.get("PYTHONPATH", "").split(os.pathsep)
                                                          if p])
    env.setdefault("OMP_NUM_THREADS", "2")
    return env


def _blob(W, H, row0, rows, epoch, board):
    return E.make_checkpoint(dict(width=W, height=H, row0=row0, epoch=epoch, topology=0, birth=8, survive=12),
                             board[row0:row0 + rows])


def test_checkpoint_roundtrip_and_reshard(tmp_path):
    W, H = 32 * 5, 23
    board = O.seed_packed(W, H, 3)
    # written by a 3-way decomposition, read back by a 2-way one
    for r0, n in [(0, 8), (8, 8), (16, 7)]:
        E.write_shard_checkpoint(str(tmp_path), _blob(W, H, r0, n, 40, board))
    assert E.complete_epochs(str(tmp_path), H) == [40]
    for r0, n in [(0, 12), (12, 11), (5, 9)]:
        h, data = E.parse_checkpoint(E.assemble_checkpoint(str(tmp_path), 40, r0, n))
        assert (h["row0"], h["rows"], h["epoch"], h["wwords"]) == (r0, n, 40, 5)
        assert (data == board[r0:r0 + n]).all()
    # an epoch missing a shard is not complete
    E.write_shard_checkpoint(str(tmp_path), _blob(W, H, 0, 8, 50, board))
    assert E.complete_epochs(str(tmp_path), H) == [40]


def _expected(W, H, gens, seed=0x5EED):
    _, h = O.run_packed(O.seed_packed(W, H, seed), W, gens, O.TORUS, O.LIFE)
    return {e + 1: int(x) for e, x in enumerate(h)}


@pytest.mark.parametrize("world,kill", [(3, (1, 25)), (2, (0, 17))])
def test_kill_backend_process_and_redeploy(tmp_path, world, kill):
    W, H, gens = 32 * 8, 60, 50
    sup = E.Supervisor(W, H, gens, world, str(tmp_path), ckpt_every=10, shard="elastic_oracle_shard:OracleShard",
                       kill=kill, timeout=240, env=_env())
    got = sup.run()
    kinds = [e["event"] for e in sup.events]
    assert kinds == ["deploy", "inject-crash", "lost", "deploy"], sup.events
    lost = sup.events[2]
    assert kill[0] in lost["ranks"] and lost["new_world"] == world - len(lost["ranks"])
    # restarted from the last complete checkpoint before the crash
    assert lost["restart_epoch"] == kill[1] // 10 * 10
    assert got == _expected(W, H, gens)


@pytest.mark.gpu
def test_kill_gpu_backend_and_respawn(gpu, tmp_path):
    """One GPU: the lost backend's board is re-spawned on the surviving GPU
    (the same one here) from the last checkpoint and replayed."""
    W, H, gens = 32 * 300, 120, 50
    sup = E.Supervisor(W, H, gens, 1, str(tmp_path), ckpt_every=10, kill=(0, 25), timeout=240, env=_env())
    got = sup.run()
    assert [e["event"] for e in sup.events] == ["deploy", "inject-crash", "lost", "deploy"], sup.events
    assert sup.events[2]["restart_epoch"] == 20
    assert got == _expected(W, H, gens)
