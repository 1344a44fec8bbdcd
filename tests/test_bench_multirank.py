"""bench.py's N > 1 path on CPU ranks with the native engine replaced by a
recorder (tests/bench_fake_runner.py; its all-reduce runs over gloo): the
path the driver's multi-GPU scaling run takes -- the communicator id through
the rendezvous file, each rank's shard, the same 65536^2 run on every rank
after its communicator exists, the settle loop every rank leaves together,
barriers, the max-over-ranks time, the per-rank diagnostics and one JSON line
from rank 0 only.  bench.py itself never imports torch."""
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


def _run(world, tmp_path, *args, extra_env=None, rc=0):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), FAKE_LOG_DIR=str(tmp_path), OMP_NUM_THREADS="1", **(extra_env or {}))
        procs.append(subprocess.Popen([sys.executable, RUNNER, "--gpus", str(world), *args], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=120) for p in procs]
    for r, (p, (o, e)) in enumerate(zip(procs, outs)):
        if rc is None:  # the watchdog tests: stopped ranks exit 4, a failed drill 3, the lost rank 0
            assert p.returncode in (0, 3, 4), e[-2000:]
        else:
            assert p.returncode == rc, e[-2000:]
    logs = [open(tmp_path / f"rank{r}.log").read().splitlines() for r in range(world)]
    return [o for o, _ in outs], logs


@pytest.mark.parametrize("world", [2, 3])
def test_multirank_bench_line(tmp_path, world):
    outs, logs = _run(world, tmp_path, "--steps", "20", "--warmup", "5", "--no-cpu", "--no-fault")
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
    settle_steps = []
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
        # seed, an untimed settle (12-generation steps), re-seed, then W
        # warm-up and exactly K timed generations on the shard, then the
        # hashed window (W + K more with hashes)
        shard = [ln for ln in log if ln.startswith(f"step 262144x{rows} ") or ln.startswith(f"seed 262144x{rows}")]
        last_seed = max(i for i, ln in enumerate(shard) if ln.startswith("seed"))
        assert [ln.split()[0] for ln in shard[:2]] == ["seed", "step"] and shard[1].split()[2] == "12"
        assert [ln.split()[2:] for ln in shard[last_seed + 1:]] == [["5"], ["20"], ["5", "hashes"], ["20", "hashes"]]
        # each rank's shard hash goes through the all-reduce
        assert [ln.split()[2] for ln in log if ln.startswith(f"hash 262144x{rows}")] == ["25", "50"]
        # every rank left the settle loop after the same number of steps
        settle_steps.append(sum(1 for ln in shard[:last_seed] if ln.startswith("step")))
        assert not any(ln.startswith("set_device") for ln in log)
    assert len(uids) == 1  # every rank joined rank 0's communicator id
    assert len(set(settle_steps)) == 1 and settle_steps[0] >= 1
    # per-rank diagnostics gathered over the ring
    for key in ("interior_ms_per_launch", "exchange_ms_per_pass", "boundary_ms_per_pass", "halo_bytes_per_pass",
                "passes", "rccl_statuses_absorbed", "hip_runtime_version", "rccl_version",
                "exchange_exposed_ms_per_pass", "pass_tail_ms_per_pass"):
        assert len(rk[key]) == world, key
    assert rk["exchange_exposed_ms_per_pass"] == [0.002] * world and rk["pass_tail_ms_per_pass"] == [0.004] * world
    assert rk["halo_bytes_per_pass"] == [2 * 2 * 12 * 262144 // 8] * world
    assert rk["exchange_ms_per_pass"] == [0.05] * world and rk["rccl_statuses_absorbed"] == [0] * world
    rt = d["runtime"]
    assert rt["same_on_all_ranks"] is True and rt["rccl_library"].startswith("/opt/rocm")
    assert rt["torch_loaded"] is False or world > 1  # the fake's all-reduce is gloo
    # parity vs tests/golden/bench_262144.json: only the sum over the ranks
    # of the shard hashes equals the golden value
    par = d["parity"]
    assert par["match"] is True, par
    whats = [(c["board"], c.get("epoch"), c.get("epochs")) for c in par["checks"]]
    # rank 0's 65536^2 windows (short, 1024-generation, single-generation passes), then the headline
    assert whats == [("65536x65536", 114, None), ("65536x65536", 1024, None), ("65536x65536", 256, None),
                     ("262144x262144", 25, None), ("262144x262144", None, [26, 50]), ("262144x262144", 50, None)]
    assert par["checks"][4]["checked"] == 25
    # the compact verdict closes the line (the driver's tail shows it)
    assert list(d)[-2:] == ["parity_failed", "parity_ok"] and d["parity_ok"] is True and d["parity_failed"] == []
    assert d["secondary"]["parity"]["match"] is True
    assert d["secondary"]["short_window"]["parity"]["epoch"] == 114
    assert d["secondary"]["single_generation_passes"]["parity"]["match"] is True


def test_multirank_bench_flags_a_wrong_shard(tmp_path):
    """A rank whose shard drifts from epoch 20 on (what a broken halo exchange
    would do) turns parity.match false, the mismatching epochs are named, the
    line closes with parity_ok false, and every rank exits non-zero after the
    line is printed."""
    outs, _ = _run(2, tmp_path, "--steps", "20", "--warmup", "5", "--no-cpu", "--no-secondary", "--no-fault",
                   extra_env={"FAKE_CORRUPT_RANK": "1"}, rc=3)
    d = json.loads([ln for ln in outs[0].splitlines() if ln.strip()][0])
    par = d["parity"]
    assert par["match"] is False
    assert par["checks"][0]["match"] is False  # epoch 25
    assert par["checks"][1]["mismatched_epochs"][:2] == [26, 27]
    assert list(d)[-1] == "parity_ok" and d["parity_ok"] is False
    assert len(d["parity_failed"]) == 3 and all("mismatch" in f for f in d["parity_failed"])


def test_single_rank_keeps_cpu_baseline_slot(tmp_path):
    """N = 1 through the same runner: the 65536^2 run comes before the whole
    board (allocation order) and no communicator is created for the headline
    run (the self-ring runs come after it)."""
    outs, logs = _run(1, tmp_path, "--steps", "12", "--warmup", "2", "--no-cpu", "--no-ring")
    d = json.loads([ln for ln in outs[0].splitlines() if ln.strip()][0])
    assert d["n_gpus"] == 1 and d["value"] > 0 and "note" not in d["secondary"]
    c1 = d["secondary"]["configs1_4096"]  # BASELINE.json configs[1], checked against golden.json
    assert c1["value"] > 0 and c1["unhashed"]["parity"]["match"] is True
    assert c1["with_state_hash"]["parity_per_generation"] == {"checked": 1000, "mismatched_epochs": [], "match": True}
    assert "tests/golden/golden.json" in d["parity"]["golden"]
    c0 = d["secondary"]["configs0_default_board"]  # BASELINE.json configs[0]'s board on this engine
    for rule in ("ref-effective", "life"):
        for mode in ("per_tick", "one_call"):
            assert c0[rule][mode]["parity"] is True and c0[rule][mode]["vs_akka_tick"] > 0
    assert d["parity"]["match"] is True
    assert [c.get("epoch") for c in d["parity"]["checks"] if c["board"] == "262144x262144"][0] == 14
    assert "ranks" not in d and d["runtime"]["torch_loaded"] is False
    log = logs[0]
    i_sec = next(i for i, ln in enumerate(log) if ln.startswith("create 65536x65536"))
    i_main = next(i for i, ln in enumerate(log) if ln.startswith("create 262144x262144"))
    assert i_sec < i_main and not any(ln.startswith("comm_init") for ln in log)


def test_single_rank_ring_windows_carry_parity(tmp_path):
    """N = 1 with the self-ring windows: the whole-board and the N = 8
    shard's windows (driver's sequence and settled) end at epoch W + K from
    the seed and are checked against bench_262144.json and
    bench_262144x32768.json; a wrong shard hash would show on its sub-line."""
    outs, logs = _run(1, tmp_path, "--steps", "20", "--warmup", "5", "--no-cpu")
    d = json.loads([ln for ln in outs[0].splitlines() if ln.strip()][0])
    ring = d["ring_schedule_n1"]
    for k in ("whole_board_self_ring", "per_rank_shard_driver_window", "per_rank_shard_self_ring"):
        assert ring[k]["parity"]["epoch"] == 25 and ring[k]["parity"]["match"] is True, k
    assert ring["per_rank_shard_self_ring"]["exchange"]["passes"] >= 1
    boards = {c["board"] for c in d["parity"]["checks"]}
    assert boards == {"7x7", "4096x4096", "65536x65536", "262144x262144", "262144x32768"}
    assert d["parity"]["match"] is True


def test_torchrun_launch_like_the_driver(tmp_path):
    """The driver's own launch form: python -m torch.distributed.run
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P
    bench.py ... (here the fake runner): the ranks find each other through
    the rendezvous file keyed by the elastic agent, and rank 0 prints the
    one line."""
    port = _free_port()
    env = dict(os.environ, FAKE_LOG_DIR=str(tmp_path), OMP_NUM_THREADS="1")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), RUNNER,
                        "--gpus", "2", "--steps", "20", "--warmup", "5", "--no-cpu", "--no-fault"],
                       env=env, capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["parity"]["match"] is True
    assert sum(d["ranks"]["rows"]) == 262144


@pytest.mark.parametrize("world", [3, 2, 5])
def test_fault_drill_sub_line(tmp_path, world):
    """configs[4] in the N > 1 bench: after the timed
    windows the ranks re-run the board from the seed with checkpoint files
    every 10 generations; rank min(3, N - 1) drops its context after
    generation 25 of 50 (its process stays up and exits 0, printing
    nothing); the rank above it restores the lost block's epoch-20 file,
    takes the 5-row light cone from its neighbours' files, replays the block
    alone and merges it with its own rows -- the fake engine refuses a blob,
    a light cone or a merge holding any other rows than the board's at that
    epoch -- and the N - 1 survivors join a new ring and step on to 50.
    Every global hash (before, replayed, at the loss, after, final) equals
    bench_262144.json, and the sub-line carries its parity and wall times."""
    outs, logs = _run(world, tmp_path, "--steps", "20", "--warmup", "5", "--no-cpu", "--no-secondary")
    d = json.loads([ln for ln in outs[0].splitlines() if ln.strip()][0])
    assert all(not o.strip() for o in outs[1:])
    f = d["fault_recovery"]
    assert f["status"] == "ok"
    victim = min(3, world - 1)
    host = victim - 1
    assert f["world_after"] == world - 1 and f["checkpoint_epoch"] == 20 and f["replayed_generations"] == 5
    assert f["parity"]["match"] is True and len(f["parity"]["checks"]) == 5
    assert f["after"]["generations"] == 25 and f["after"]["value"] > 0 and f["recovery_ms"] >= 0
    assert d["parity_ok"] is True and d["parity"]["match"] is True
    whats = [c["what"] for c in d["parity"]["checks"] if c["what"].startswith("fault drill")]
    assert len(whats) == 5
    H = 262144
    for r, log in enumerate(logs):
        i_seed = max(i for i, ln in enumerate(log) if ln.startswith("seed 262144x"))
        drill = log[i_seed:]
        ev = [ln.split()[0] for ln in drill]
        assert [ln.split()[3] for ln in drill if ln.startswith("checkpoint")] == ["10", "20"]
        assert "comm_abort" in ev
        if r == victim:  # drops everything after generation 25: no further step, ring or hash
            i_abort = ev.index("comm_abort")
            assert ev[i_abort + 1:] == ["close"], drill[i_abort:]
            continue
        comm = [ln.split() for ln in drill if ln.startswith("comm_init")]
        assert [c[2:] for c in comm] == [[str(r if r < victim else r - 1), str(world - 1)]]
        if r == host:
            v0 = victim * (H // world) + min(victim, H % world)
            vn = H // world + (1 if victim < H % world else 0)
            assert f"restore 262144x{vn} {v0} 20" in drill and f"replay 262144x{vn} {v0} 20 5" in drill
            mine = H // world + (1 if host < H % world else 0)
            assert any(ln.startswith(f"create 262144x{mine + vn} ") for ln in drill)
            assert any(ln.startswith(f"restore 262144x{mine + vn} ") and ln.endswith(" 25") for ln in drill)
        steps = [ln.split()[2] for ln in drill if ln.startswith("step 262144x") and "x%d " % vn not in ln] \
            if r == host else [ln.split()[2] for ln in drill if ln.startswith("step 262144x")]
        assert steps[-1] == "25"


def test_fault_drill_watchdog(tmp_path):
    """A ring rebuild that never completes must not cost the measured line:
    past --fault-timeout every rank stops (exit 4), rank 0 having printed the
    line with fault_recovery marked timed out and parity_ok false."""
    outs, _ = _run(3, tmp_path, "--steps", "20", "--warmup", "5", "--no-cpu", "--no-secondary",
                   "--fault-timeout", "8", extra_env={"FAKE_HANG_REJOIN": "1"}, rc=None)
    d = json.loads([ln for ln in outs[0].splitlines() if ln.strip()][0])
    assert d["value"] > 0 and d["parity"]["match"] is True  # the measured windows are intact
    fr = d["fault_recovery"]
    assert (fr["status"], fr["timeout_s"]) == ("timed out", 8.0) and "stderr" in fr["note"]
    assert "rank_errors" not in fr  # a hang, not an exception
    # the line is the snapshot taken before the drill: none of its checks leaked in
    assert not any("fault drill" in c["what"] for c in d["parity"]["checks"])
    assert d["parity_ok"] is False and any("fault drill" in f for f in d["parity_failed"])


def test_fault_drill_skips_without_room(tmp_path):
    """No directory with room for the checkpoint files: every rank skips the
    drill together (rank 0 decides), the line says so, and the measured
    windows stand (exit 0)."""
    outs, logs = _run(2, tmp_path, "--steps", "20", "--warmup", "5", "--no-cpu", "--no-secondary",
                      extra_env={"FAKE_NO_ROOM": "1"})
    d = json.loads([ln for ln in outs[0].splitlines() if ln.strip()][0])
    assert d["fault_recovery"]["status"] == "skipped" and d["parity_ok"] is True
    assert not any(ln.startswith("comm_abort") for log in logs for ln in log)


def test_fault_drill_error_on_rank0(tmp_path):
    """A drill that fails on rank 0 (a checkpoint write raising) still gets
    the measured line out: status error, parity_ok false, exit 3 on rank 0;
    the peers, left waiting in a collective, stop at the watchdog (exit 4)."""
    outs, _ = _run(3, tmp_path, "--steps", "20", "--warmup", "5", "--no-cpu", "--no-secondary",
                   "--fault-timeout", "8", extra_env={"FAKE_DRILL_RAISE": "0"}, rc=None)
    d = json.loads([ln for ln in outs[0].splitlines() if ln.strip()][0])
    assert d["fault_recovery"]["status"] == "error" and "No space left" in d["fault_recovery"]["error"]
    assert d["value"] > 0 and d["parity_ok"] is False


def test_fault_drill_error_on_a_peer(tmp_path):
    """A drill that raises on a non-zero rank (its checkpoint write at epoch
    20) leaves rank 0 in a collective the peer never joins: with RCCL it
    waits for the watchdog, with the gloo stand-in the collective breaks when
    the peer exits (and a third rank's collective may break with it, so it
    can be named too).  Either way rank 0's line names the peer's exception
    under fault_recovery.rank_errors and fails parity."""
    outs, _ = _run(3, tmp_path, "--steps", "20", "--warmup", "5", "--no-cpu", "--no-secondary",
                   "--fault-timeout", "8", extra_env={"FAKE_DRILL_RAISE": "1"}, rc=None)
    d = json.loads([ln for ln in outs[0].splitlines() if ln.strip()][0])
    fr = d["fault_recovery"]
    assert fr["status"] in ("timed out", "error") and "1" in fr["rank_errors"] and "0" not in fr["rank_errors"]
    assert "No space left" in fr["rank_errors"]["1"]
    assert d["parity_ok"] is False
