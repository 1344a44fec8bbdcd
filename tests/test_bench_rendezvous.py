"""bench.py's torch-free rendezvous (CPU): rank 0's RCCL unique id travels
through a file keyed by MASTER_ADDR:MASTER_PORT; a rank ignores a file older
than its own start (minus two minutes of launch skew) -- the leftover of an
earlier job on the same port -- and rank 0 removes the file once every rank
has joined (after the first barrier over the new communicator)."""
import os
import threading
import time
import types

import bench


class _Eng:
    def __init__(self):
        self.joined = None
        self.reduced = 0

    def comm_init(self, uid, rank, world):
        self.joined = (uid, rank, world)

    def allreduce_u64(self, values):
        self.reduced += 1
        return values


_N = types.SimpleNamespace(GOL_UNIQUE_ID_BYTES=128, unique_id=lambda: bytes(range(128)))


def _job(monkeypatch, rank, port):
    monkeypatch.setenv("RANK", str(rank))
    monkeypatch.setenv("LOCAL_RANK", str(rank))
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(port))
    return bench.Job(2)


def test_rank0_publishes_then_removes(monkeypatch):
    job = _job(monkeypatch, 0, 41001)
    eng = _Eng()
    path = job.uid_path()
    job.join(eng, _N)
    assert eng.joined == (bytes(range(128)), 0, 2) and eng.reduced == 1  # the barrier
    assert not os.path.exists(path)


def test_stale_file_is_ignored(monkeypatch):
    job = _job(monkeypatch, 1, 41002)
    path = job.uid_path()
    with open(path, "wb") as f:
        f.write(b"\x01" * 128)
    old = time.time() - 3600
    os.utime(path, (old, old))
    fresh = bytes(range(128, 256))

    def publish():
        time.sleep(0.3)
        tmp = path + ".tmp"
        with open(tmp, "wb") as f:
            f.write(fresh)
        os.replace(tmp, path)

    t = threading.Thread(target=publish)
    t.start()
    eng = _Eng()
    job.join(eng, _N, timeout=20)
    t.join()
    assert eng.joined == (fresh, 1, 2)
    os.unlink(path)


def test_gather_lays_rows_by_rank(monkeypatch):
    job = _job(monkeypatch, 1, 41003)

    class Sum(_Eng):
        def allreduce_u64(self, values):
            import numpy as np
            v = np.asarray(values, dtype=np.uint64).copy()
            v[:3] += np.array([7, 8, 9], dtype=np.uint64)  # rank 0's row
            return v

    job.eng = Sum()
    assert job.gather([1, 2, 3]) == [[7, 8, 9], [1, 2, 3]]


def test_torchrun_key_names_the_agent(monkeypatch):
    """Under torch.distributed.run (TORCHELASTIC_RUN_ID set) the file name
    also carries the ranks' common parent, the elastic agent: a file a
    crashed earlier torchrun job on the same port left is never read."""
    job = _job(monkeypatch, 1, 41010)
    plain = job.uid_path()
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "none")
    here = job.uid_path()
    monkeypatch.setattr(os, "getppid", lambda: 1)
    other_agent = job.uid_path()
    assert len({plain, here, other_agent}) == 3


def test_launch_key_outside_torchrun(monkeypatch):
    """Outside torch.distributed.run the key carries the ranks' common parent
    too (address + port alone let a crashed earlier job's file be
    read), or GOL_BENCH_RUN_ID when the launcher names the launch; a later
    ring of the same job (the fault drill's) has its own file."""
    monkeypatch.delenv("TORCHELASTIC_RUN_ID", raising=False)
    monkeypatch.delenv("GOL_BENCH_RUN_ID", raising=False)
    job = _job(monkeypatch, 1, 41011)
    here = job.uid_path()
    assert job.uid_path("fault") != here
    monkeypatch.setattr(os, "getppid", lambda: 1)
    other_parent = job.uid_path()
    monkeypatch.setenv("GOL_BENCH_RUN_ID", "launch-a")
    a = job.uid_path()
    monkeypatch.setattr(os, "getppid", lambda: 2)
    assert job.uid_path() == a  # an explicit launch id does not depend on the parent
    monkeypatch.setenv("GOL_BENCH_RUN_ID", "launch-b")
    assert len({here, other_parent, a, job.uid_path()}) == 4


def test_multi_node_launch_fails_fast(monkeypatch):
    """The file rendezvous serves one node: WORLD_SIZE > LOCAL_WORLD_SIZE
    stops with a message instead of waiting for a file no other node sees."""
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    try:
        _job(monkeypatch, 0, 41012)
    except SystemExit as e:
        assert "one node" in str(e)
    else:
        raise AssertionError("a 2-node launch was accepted")


def test_later_ring_joins_with_its_own_rank(monkeypatch):
    """join(tag=..., rank=..., world=...): the fault drill's N - 1 ring, with
    the survivors renumbered; the job's own engine is left alone."""
    job = _job(monkeypatch, 0, 41013)
    first, later = _Eng(), _Eng()
    job.join(first, _N)
    job.join(later, _N, tag="fault", rank=0, world=1)
    assert later.joined == (bytes(range(128)), 0, 1) and later.reduced == 0  # a 1-rank ring needs no barrier
    assert job.eng is first
