"""Cross-process fault path (gameoflife.elastic, BASELINE.json config 5):
checkpoint files, light-cone rows, and the supervisor crashing backend
processes mid-run -- once, and recurrently on the reference's errors.delay /
errors.every / max-crashes schedule -- with lost-shard-only recovery (the
block is re-spawned next to a survivor and replayed alone; nobody rolls
back).  The CPU tests run real backend processes with the oracle/gloo shard
double (tests/elastic_oracle_shard.py); the GPU tests run libgol backends."""
import os

import numpy as np
import pytest

from gameoflife import elastic as E
from gameoflife.board import SimulationParams, crash_schedule
from oracle import oracle as O

TESTS = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(TESTS)
ORACLE_SHARD = "elastic_oracle_shard:OracleShard"


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
    assert E.covering_epochs(str(tmp_path), 0, 8) == [40, 50]
    # overlapping blocks of two decompositions at one epoch (a merged block
    # next to the blocks it replaced) hold the same rows: still complete
    E.write_shard_checkpoint(str(tmp_path), _blob(W, H, 0, 16, 40, board))
    assert E.complete_epochs(str(tmp_path), H) == [40]
    assert (E.parse_checkpoint(E.assemble_checkpoint(str(tmp_path), 40, 3, 20))[1] == board[3:23]).all()


def test_checkpoint_rows_reads_any_row_list(tmp_path):
    """checkpoint_rows seeks to runs of consecutive rows: any row list --
    unsorted, repeated, wrapping, across files of two decompositions -- comes
    back as those rows of the board; rows no file holds, and a file whose
    header disagrees with its name, are refused."""
    W, H = 32 * 3, 41
    board = O.seed_packed(W, H, 11)
    rng = np.random.default_rng(7)
    for epoch in range(6):
        d = str(tmp_path / f"c{epoch}")
        cuts = sorted(set(rng.integers(1, H, size=int(rng.integers(0, 6))).tolist()))
        for r0, r1 in zip([0] + cuts, cuts + [H]):
            E.write_shard_checkpoint(d, _blob(W, H, r0, r1 - r0, epoch, board))
        if epoch % 2:  # a merged block overlapping the others
            E.write_shard_checkpoint(d, _blob(W, H, 5, 20, epoch, board))
        for _ in range(8):
            idx = rng.integers(0, H, size=int(rng.integers(1, 3 * H))).tolist()
            if rng.random() < 0.5:
                a = int(rng.integers(0, H))
                idx = [(a + k) % H for k in range(int(rng.integers(1, H)))]  # a wrapping run
            assert (E.checkpoint_rows(d, epoch, idx) == board[idx]).all()
    d = str(tmp_path / "gap")
    E.write_shard_checkpoint(d, _blob(W, H, 0, 10, 0, board))
    E.write_shard_checkpoint(d, _blob(W, H, 12, 29, 0, board))
    assert (E.checkpoint_rows(d, 0, [9, 12]) == board[[9, 12]]).all()
    with pytest.raises(FileNotFoundError):
        E.checkpoint_rows(d, 0, [9, 10])
    os.replace(os.path.join(E.epoch_dir(d, 0), "r0000000000_10.gol"),
               os.path.join(E.epoch_dir(d, 0), "r0000000010_10.gol"))
    with pytest.raises(ValueError):
        E.checkpoint_rows(d, 0, [11])


def test_light_cone_rows(tmp_path):
    W, H = 32 * 3, 20
    board = O.seed_packed(W, H, 8)
    for r0, n in [(0, 7), (7, 7), (14, 6)]:
        E.write_shard_checkpoint(str(tmp_path), _blob(W, H, r0, n, 10, board))
    up, dn = E.light_cone(str(tmp_path), 10, 7, 7, 3, H, torus=True)
    assert (up == board[4:7]).all() and (dn == board[14:17]).all()
    up, dn = E.light_cone(str(tmp_path), 10, 0, 7, 9, H, torus=True)  # wraps, deeper than a shard
    assert (up == board[[11, 12, 13, 14, 15, 16, 17, 18, 19]]).all() and (dn == board[7:16]).all()
    up, dn = E.light_cone(str(tmp_path), 10, 14, 6, 4, H, torus=False)  # clipped: dead beyond the edge
    assert (up == board[10:14]).all() and (dn == 0).all()
    # a block stepped with its light cone (torus in x, garbage ends) matches
    # the whole board stepped the same number of generations
    d = 5
    up, dn = E.light_cone(str(tmp_path), 10, 7, 7, d, H, torus=True)
    ext = np.vstack([up, board[7:14], dn])
    for _ in range(d):
        ext = O.step_packed(ext, W)
    ref, _ = O.run_packed(board, W, d, want_hashes=False)
    assert (ext[d:d + 7] == ref[7:14]).all()


def test_recovery_epoch_needs_the_light_cone(tmp_path):
    """a backend killed at a checkpoint epoch never writes
    that epoch's file, so its neighbour's own rows may be on disk at an epoch
    whose light cone is not.  recovery_epoch goes back to an epoch holding the
    block and its epoch - c rows on each side (mod H on a torus)."""
    W, H = 32 * 4, 60
    board = O.seed_packed(W, H, 5)
    for r0, n in [(0, 20), (20, 20), (40, 20)]:
        E.write_shard_checkpoint(str(tmp_path), _blob(W, H, r0, n, 0, board))
    for r0, n in [(0, 20), (40, 20)]:  # rows 20..39 died at epoch 10 before writing
        E.write_shard_checkpoint(str(tmp_path), _blob(W, H, r0, n, 10, board))
    d = str(tmp_path)
    assert E.covering_epochs(d, 40, 60) == [0, 10]
    assert E.recovery_epoch(d, 40, 60, 10, H, torus=True) == 10  # no light cone needed
    assert E.recovery_epoch(d, 40, 60, 15, H, torus=True) == 0   # rows 35..39 missing at 10
    assert E.recovery_epoch(d, 0, 20, 12, H, torus=True) == 0    # rows 20, 21 missing at 10
    assert E.recovery_epoch(d, 45, 55, 15, H, torus=True) == 10  # cone [40, 60) is on disk
    assert E.recovery_epoch(d, 40, 60, 15, H, torus=False) == 0
    assert E.light_cone_ranges(50, 58, 5, H, True) == [(45, 60), (0, 3)]
    assert E.light_cone_ranges(2, 10, 5, H, True) == [(57, 60), (0, 15)]
    assert E.light_cone_ranges(0, 60, 3, H, True) == [(0, 60)]
    assert E.light_cone_ranges(2, 10, 5, H, False) == [(0, 15)]


def test_neighbour_lost_after_a_crash_at_a_checkpoint_epoch(tmp_path):
    """The ADVICE r02 scenario end to end: 3 backends on a torus, one crashed
    at epoch 10 (= ckpt_every: it dies before writing e10), then the backend
    next to the merged block crashed at 15, before the next checkpoint.  Every
    generation's hash equals the uninterrupted oracle run."""
    W, H, gens = 32 * 6, 60, 30
    sup = E.Supervisor(W, H, gens, 3, str(tmp_path), ckpt_every=10, shard=ORACLE_SHARD,
                       crashes=[(10, 1), (15, 1)], chunk=5, timeout=300, env=_env())
    got = sup.run()
    lost = [e for e in sup.events if e["event"] == "lost"]
    assert [(e["rows"], e["epoch"]) for e in lost] == [([20, 40], 10), ([40, 60], 15)]
    assert lost[0]["checkpoint_epoch"] == 0 and lost[1]["checkpoint_epoch"] == 10
    assert got == _expected(W, H, gens)


def test_demo_cli_eight_backends_kill_3_at_25(tmp_path):
    """`python -m gameoflife.elastic demo --world 8 --kill 3@25` -- the config-5
    control flow with 8 backend processes (the oracle double, gloo ring): the
    faulted run's hashes equal the uninterrupted run's at every generation."""
    import json
    import subprocess
    import sys
    out = subprocess.run([sys.executable, "-m", "gameoflife.elastic", "demo", "--width", "256", "--height", "96",
                          "--gens", "50", "--every", "10", "--world", "8", "--kill", "3@25",
                          "--workdir", str(tmp_path / "run"), "--shard", ORACLE_SHARD],
                         env=dict(_env(), PYTHONPATH=os.pathsep.join([os.path.join(ROOT, "akka-game-of-life_amd"),
                                                                       _env()["PYTHONPATH"]])),
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads(out.stdout.strip().splitlines()[-1])
    assert d["hashes_equal"] is True and d["generations"] == 50
    lost = [e for e in d["events"] if e["event"] == "lost"]
    assert len(lost) == 1 and lost[0]["epoch"] == 25 and lost[0]["checkpoint_epoch"] == 20
    assert lost[0]["rows"] == [36, 48] and lost[0]["new_world"] == 7
    ref = _expected(256, 96, 50)
    got = E.Supervisor.__new__(E.Supervisor)
    got.workdir = str(tmp_path / "run")
    assert got.hashes() == ref


def test_crash_schedule_follows_reference_keys():
    """BoardCreator.scala:97-108 timing: ticks at start + k * tick advance to
    epoch k + 1; crash i at delay + i * every, at most max-crashes."""
    p = SimulationParams(start_delay_ms=1000, tick_ms=3000, first_error_after_ms=10000, error_every_ms=15000,
                         max_number_of_crashes=100)
    assert [g for g, _ in crash_schedule(p, 30)] == [4, 9, 14, 19, 24, 29]
    p2 = SimulationParams(start_delay_ms=0, tick_ms=1000, first_error_after_ms=7000, error_every_ms=9000,
                          max_number_of_crashes=2)
    assert [g for g, _ in crash_schedule(p2, 100)] == [8, 17]
    assert crash_schedule(p2, 100, seed=5) == crash_schedule(p2, 100, seed=5)


def _expected(W, H, gens, seed=0x5EED):
    _, h = O.run_packed(O.seed_packed(W, H, seed), W, gens, O.TORUS, O.LIFE)
    return {e + 1: int(x) for e, x in enumerate(h)}


@pytest.mark.parametrize("world,kill", [(3, (1, 25)), (2, (0, 17))])
def test_kill_backend_process_and_respawn_alone(tmp_path, world, kill):
    W, H, gens = 32 * 8, 60, 50
    sup = E.Supervisor(W, H, gens, world, str(tmp_path), ckpt_every=10, shard=ORACLE_SHARD,
                       kill=kill, timeout=240, env=_env())
    got = sup.run()
    kinds = [e["event"] for e in sup.events]
    assert kinds == ["deploy", "inject-crash", "lost"], sup.events
    lost = sup.events[2]
    # only the lost block replays, from its last checkpoint; the others stay
    assert lost["checkpoint_epoch"] == kill[1] // 10 * 10 and lost["epoch"] == kill[1]
    assert lost["replayed_generations"] == kill[1] % 10 and lost["new_world"] == world - 1
    assert "absorbed_by" in lost
    assert got == _expected(W, H, gens)


def test_recurring_crashes_on_the_reference_schedule(tmp_path):
    """errors.delay / errors.every / max-crashes drive repeated crashes: 3
    backends shrink to 1, then the last one dies twice and is re-spawned from
    the checkpoint files alone; every generation's hash equals the
    uninterrupted oracle run."""
    W, H, gens = 32 * 6, 45, 48
    p = SimulationParams(start_delay_ms=0, tick_ms=1000, first_error_after_ms=6000, error_every_ms=11000,
                         max_number_of_crashes=4)
    crashes = crash_schedule(p, gens, seed=3)
    assert [g for g, _ in crashes] == [7, 18, 29, 40]
    sup = E.Supervisor(W, H, gens, 3, str(tmp_path), ckpt_every=5, shard=ORACLE_SHARD, crashes=crashes,
                       chunk=3, timeout=400, env=_env())
    got = sup.run()
    lost = [e for e in sup.events if e["event"] == "lost"]
    assert len(lost) == 4
    assert [e["new_world"] for e in lost] == [2, 1, 1, 1]
    assert "respawned_as" in lost[2] and "respawned_as" in lost[3]
    assert got == _expected(W, H, gens)


@pytest.mark.gpu
def test_kill_gpu_backend_and_respawn(gpu, tmp_path):
    """One GPU, one backend crashed three times: each time a fresh backend
    restores the board from the checkpoint files and replays the lost
    generations alone (gol_replay on the whole torus: the light cone wraps)."""
    W, H, gens = 32 * 300, 120, 50
    sup = E.Supervisor(W, H, gens, 1, str(tmp_path), ckpt_every=10, crashes=[(13, 0), (25, 0), (40, 0)],
                       chunk=4, timeout=400, env=_env())
    got = sup.run()
    lost = [e for e in sup.events if e["event"] == "lost"]
    assert [(e["checkpoint_epoch"], e["epoch"]) for e in lost] == [(10, 13), (20, 25), (30, 40)]
    assert got == _expected(W, H, gens)
