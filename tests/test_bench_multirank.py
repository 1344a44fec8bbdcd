"""bench.py's N > 1 path on CPU ranks (gloo) with the native engine replaced
by a recorder (tests/bench_fake_runner.py): the path the driver's multi-GPU
scaling run takes -- communicator-id broadcast, each rank's shard, the same
65536^2 run on every rank after its communicator exists, barriers, the
max-over-ranks time and one JSON line from rank 0 only."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUNNER = os.path.join(ROOT, "tests", "bench_fake_runner.py")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world, tmp_path, *args, extra_env=None):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), FAKE_LOG_DIR=str(tmp_path), OMP_NUM_THREADS="1", **(extra_env or {}))
        procs.append(subprocess.Popen([sys.executable, RUNNER, "--gpus", str(world), *args], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=120) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
    logs = [open(tmp_path / f"rank{r}.log").read().splitlines() for r in range(world)]
    return [o for o, _ in outs], logs


@pytest.mark.parametrize("world", [2, 3])
def test_multirank_bench_line(tmp_path, world):
    outs, logs = _run(world, tmp_path, "--steps", "20", "--warmup", "5", "--no-cpu")
    lines = [ln for ln in outs[0].splitlines() if ln.strip()]
    assert len(lines) == 1, outs[0]
    assert all(not o.strip() for o in outs[1:])  # only rank 0 prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["steps"] == 20 and d["warmup"] == 5
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["scaling"] == "strong"
    assert f"x{world}" in d["config"]["parallelism"]
    assert d["roofline"]["bound"] == "valu"
    assert "cpu_baseline" not in d  # rank 0 at N = 1 only
    assert "note" in d["secondary"] and d["secondary"]["value"] > 0
    rk = d["ranks"]
    assert len(rk["ms_per_step"]) == world and sum(rk["rows"]) == 262144
    assert abs(max(rk["ms_per_step"]) - d["ms_per_step"]) < 1e-3
    uids = set()
    H = 262144
    for r, log in enumerate(logs):
        ev = [ln.split()[0] for ln in log]
        # the shard and its communicator first, then the 65536^2 run, then the timed shard run
        i_comm = ev.index("comm_init")
        i_sec = next(i for i, ln in enumerate(log) if ln.startswith("create 65536x65536"))
        assert i_comm < i_sec
        seeds = [i for i, ln in enumerate(log) if ln.startswith("seed 262144x")]
        assert seeds and seeds[0] > i_sec
        rows = H // world + (1 if r < H % world else 0)
        assert any(ln.startswith(f"create 262144x{rows} ") for ln in log)
        uids.add(next(ln for ln in log if ln.startswith("comm_init")).split()[1])
        comm = next(ln for ln in log if ln.startswith("comm_init")).split()
        assert comm[2:] == [str(r), str(world)]
        # W warm-up then exactly K timed generations on the shard
        shard_steps = [int(ln.split()[2]) for ln in log if ln.startswith(f"step 262144x{rows} ")]
        assert shard_steps[:2] == [5, 20]
        # then the hashed window (W + K more generations with hashes), and each
        # rank's shard hash goes through the all-reduce
        assert [ln.split()[2:] for ln in log if ln.startswith(f"step 262144x{rows} ")][2:4] == \
            [["5", "hashes"], ["20", "hashes"]]
        assert [ln.split()[2] for ln in log if ln.startswith(f"hash 262144x{rows}")] == ["25", "50"]
        assert sum(1 for ln in log if ln.startswith("allreduce")) == 3
    assert len(uids) == 1  # every rank joined rank 0's communicator id
    # parity vs tests/golden/bench_262144.json: only the sum over the ranks
    # of the shard hashes equals the golden value
    par = d["parity"]
    assert par["match"] is True, par
    whats = [(c.get("epoch"), c.get("epochs")) for c in par["checks"]]
    assert whats == [(25, None), (None, [26, 50]), (50, None)]
    assert par["checks"][1]["checked"] == 25


def test_multirank_bench_flags_a_wrong_shard(tmp_path):
    """A rank whose shard drifts from epoch 20 on (what a broken halo exchange
    would do) turns parity.match false, and the mismatching epochs are named."""
    outs, _ = _run(2, tmp_path, "--steps", "20", "--warmup", "5", "--no-cpu", "--no-secondary",
                   extra_env={"FAKE_CORRUPT_RANK": "1"})
    d = json.loads([ln for ln in outs[0].splitlines() if ln.strip()][0])
    par = d["parity"]
    assert par["match"] is False
    assert par["checks"][0]["match"] is False  # epoch 25
    assert par["checks"][1]["mismatched_epochs"][:2] == [26, 27]


def test_single_rank_keeps_cpu_baseline_slot(tmp_path):
    """N = 1 through the same runner: the 65536^2 run comes before the whole
    board (allocation order) and no communicator is created for the headline
    run (the self-ring runs come after it)."""
    outs, logs = _run(1, tmp_path, "--steps", "12", "--warmup", "2", "--no-cpu", "--no-ring")
    d = json.loads([ln for ln in outs[0].splitlines() if ln.strip()][0])
    assert d["n_gpus"] == 1 and d["value"] > 0 and "note" not in d["secondary"]
    assert d["parity"]["match"] is True and d["parity"]["checks"][0]["epoch"] == 14
    log = logs[0]
    i_sec = next(i for i, ln in enumerate(log) if ln.startswith("create 65536x65536"))
    i_main = next(i for i, ln in enumerate(log) if ln.startswith("create 262144x262144"))
    assert i_sec < i_main and not any(ln.startswith("comm_init") for ln in log)
