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


def _run(world, tmp_path, *args):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), FAKE_LOG_DIR=str(tmp_path), OMP_NUM_THREADS="1")
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
    assert len(uids) == 1  # every rank joined rank 0's communicator id


def test_single_rank_keeps_cpu_baseline_slot(tmp_path):
    """N = 1 through the same runner: the 65536^2 run comes before the whole
    board (allocation order) and no communicator is created for the headline
    run (the self-ring runs come after it)."""
    outs, logs = _run(1, tmp_path, "--steps", "12", "--warmup", "2", "--no-cpu", "--no-ring")
    d = json.loads([ln for ln in outs[0].splitlines() if ln.strip()][0])
    assert d["n_gpus"] == 1 and d["value"] > 0 and "note" not in d["secondary"]
    log = logs[0]
    i_sec = next(i for i, ln in enumerate(log) if ln.startswith("create 65536x65536"))
    i_main = next(i for i, ln in enumerate(log) if ln.startswith("create 262144x262144"))
    assert i_sec < i_main and not any(ln.startswith("comm_init") for ln in log)
