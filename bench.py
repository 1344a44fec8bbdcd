#!/usr/bin/env python3
"""bench.py -- generation-step throughput (GCUPS) and its roofline.

Workload (BASELINE.json configs[3], DESIGN.md "Measurement"): a 262144 x
262144 torus, B3/S23, Bernoulli(0.5) splitmix64 board (seed 0x5EED),
row-sharded over N GPUs (strong scaling; N = 1 runs the whole board on one
GPU).  A "step" is one generation of the whole board.  Every GPU also runs
the single-GPU roofline case of configs[2] (65536^2) before the timed
262144^2 window -- the same sequence at every N -- and rank 0 reports it
under "secondary".

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

value = W*H*K / max-over-ranks wall time of the K timed generations (GCUPS),
with the board already resident in HBM.  Before its W warm-up steps every
timed board is seeded, stepped untimed for a short settle (the chip's clock
recovers over ~20 launches after an idle gap such as the 16 GiB allocation,
profiles/r02_warmup_curve.txt) and re-seeded, so the timed epochs are W + K
from the seed and every window's hash is checked against a committed golden
table (tests/golden/bench_*.json).

No torch: the process is one rank of the launcher (RANK / WORLD_SIZE /
LOCAL_RANK from the environment), the RCCL unique id travels through a file
keyed by MASTER_ADDR:MASTER_PORT and the launcher's pid, and the barriers and
the max over ranks are gol_comm_allreduce_u64 calls on the shard's own
communicator -- so libgol runs on the same HIP runtime and RCCL (/opt/rocm's)
as the pytest GPU suite and a JVM host; the line's "runtime" field names them.

roofline: the dominant kernel (the whole-shard launch at
N = 1, a shard's interior-rows launch at N > 1) is bound by VALU issue, not by
HBM -- temporal blocking fuses 6-8 generations per pass over the plane.  So:
  * roofline.bound = "valu": achieved = cell-updates per second of that launch
    (cells x generations per launch / its mean HIP-event duration), peak = the
    VALU-issue ceiling of the kernel's loop mix at the guide's 2.4 GHz max
    clock, frac = achieved / peak; roofline.held_clock prices the same launches
    at the clock they actually held (in-kernel probe, gol_profile_clock) as an
    issue-efficiency diagnostic, with the PMC clock (profiles/) beside it;
  * roofline.frac_guide_issue prices the same launches at the guide's 2 cycles
    per wave64 VALU instruction (MI355X_MICROARCH.md) instead of the measured
    per-op costs, and roofline.issue_rate gives the wave-VALU instructions per
    cycle per SIMD the launches issued (0.5 = that ceiling);
  * roofline.copy_peak = the measured stream-copy peak (profiles/copy_peak.json,
    scripts/micro/copy_bw.hip); single-generation lines add frac_of_copy_peak;
  * roofline.traffic = PMC HBM bytes per launch, and roofline.hbm the physical
    HBM bandwidth that implies against the 8 TB/s spec;
  * roofline.hbm_effective = SURVEY.md section 8(d)'s 2 bits per cell-update,
    counted per generation: above 1 by construction of temporal blocking.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BYTES_PER_CELL_UPDATE = 0.25
CLOCK_MAX_GHZ = 2.4  # MI355X_MICROARCH.md max clock
SIMDS = 256 * 4
CELLS_PER_WAVE_INSTR = 64 * 32  # 64 lanes x one 32-cell word
DEFAULT_GPP = 0  # generations per HBM pass: 0 = libgol's pass planner (gol_pass_plan, DESIGN.md "Pass planner")

# Issue-cost model of the multi-generation kernel's loop (DESIGN.md "Roofline"):
# VALU instructions per 32-cell word and generation of multistep_hg_kernel<2, G,
# LIFE> on the pair layout and the measured cycles per wave64 instruction on one
# SIMD (profiles/r01_valu_op_costs.txt).  Round 4's row-pair-shared circuit
# (gol_stencil.h rule_b3s23_pair): per word-generation 2 bitop3 for the row's
# horizontal sum, half of the pair sum P (1 bitop3 + 1 v_xor + 1 v_and per two
# rows) and a 4-bitop3 tail, plus one funnel shift and one DPP move
# (scripts/isa_loop.py census of the G = 12 loop: 6.54 bitop3 and
# 0.47 v_xor + 0.47 v_and per v_alignbit, the (G + 1) / G arrivals included).
VALU_MIX = {"v_bitop3_b32": (7, 2.3), "v_xor_b32": (0.5, 2.3), "v_and_b32": (0.5, 2.3),
            "v_alignbit_b32": (1, 4.1), "v_mov_b32_dpp": (1, 4.3)}
# The fused hash adds one v_mad_u64_u32 per word and generation (DESIGN.md "State hash").
VALU_MIX_HASH = dict(VALU_MIX, v_mad_u64_u32=(1, 4.6))
# MI355X_MICROARCH.md (CU / SIMD model): a wave64 VALU instruction issues over
# 2 cycles on its SIMD -- the guide's rate, which prices frac_guide_issue
# whatever the instructions are (the mix-priced frac uses the measured per-op
# costs above instead).
GUIDE_CYCLES_PER_VALU = 2.0
COPY_PEAK_FILE = os.path.join("profiles", "copy_peak.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: 60 timed generations = 6 x 10 passes at 262144^2 (the planner's choice)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=6)
    ap.add_argument("--board", type=int, default=262144, help="board edge (cells)")
    ap.add_argument("--band", type=int, default=0, help="rows per band (0 = auto)")
    ap.add_argument("--gpp", type=int, default=DEFAULT_GPP,
                    help="generations fused per HBM pass (temporal blocking depth 1..12; 0 = automatic)")
    ap.add_argument("--hash", action="store_true", help="fuse the per-generation state hash")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--no-ring", action="store_true", help="skip the N = 1 ring-schedule measurements")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-fault", action="store_true",
                    help="skip the N > 1 fault drill (config 5: a rank lost at generation 25 of 50, its shard "
                         "re-spawned on a surviving GPU)")
    ap.add_argument("--fault-timeout", type=float, default=240.0,
                    help="seconds the fault drill may take before every rank gives up on it (the line is then "
                         "printed without it, parity_ok false)")
    ap.add_argument("--allow-unchecked", action="store_true",
                    help="exit 0 when a window has no golden value (boards without a table); a mismatch still fails")
    return ap.parse_args()


class Job:
    """This process's place in the launch (one process per GPU, one node).

    Ranks come from the launcher's environment (torch.distributed.run sets
    RANK, WORLD_SIZE, LOCAL_RANK, LOCAL_WORLD_SIZE, MASTER_ADDR, MASTER_PORT).
    Rank 0's RCCL unique id reaches the other ranks through a file in the
    node's temp directory named after MASTER_ADDR:MASTER_PORT and the launch:
    the ranks' common parent (torch.distributed.run's elastic agent, or
    whatever started them) or GOL_BENCH_RUN_ID when set, so a file a crashed
    earlier job left behind on the same port is never read; a file older than
    this rank's start (minus two minutes of launch skew) is ignored as well.
    After the first barrier over the new communicator every rank has read it,
    and rank 0 removes it.  Barriers and the max over ranks are
    gol_comm_allreduce_u64 calls on the shard's own RCCL communicator: no
    torch, no second collective library."""

    def __init__(self, n):
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world != n:
            raise SystemExit(f"--gpus {n} but WORLD_SIZE={self.world}")
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(self.world)))
        if self.world > local_world:
            raise SystemExit(f"WORLD_SIZE={self.world} > LOCAL_WORLD_SIZE={local_world}: bench.py's rendezvous "
                             "(a file in this node's temp directory) serves one node only")
        self.eng = None  # the engine whose communicator carries the collectives
        self.t_start = time.time()

    def uid_path(self, tag=""):
        # The launch key: under torch.distributed.run every local rank is a
        # child of the same elastic agent (its run id is "none" unless
        # --rdzv-id is given); other launchers' ranks share their launcher as
        # parent too, unless GOL_BENCH_RUN_ID names the launch explicitly.
        launch = os.environ.get("GOL_BENCH_RUN_ID") or f"{os.environ.get('TORCHELASTIC_RUN_ID', '')}_{os.getppid()}"
        key = "_".join([os.environ.get("MASTER_ADDR", "127.0.0.1"), os.environ.get("MASTER_PORT", "0"), launch, tag])
        return os.path.join(tempfile.gettempdir(), "gol_bench_uid_" + hashlib.sha1(key.encode()).hexdigest()[:16])

    def join(self, eng, N, timeout=300.0, tag="", rank=None, world=None):
        """Attach `eng` to the job's RCCL ring (rank 0 makes the id); `tag`,
        `rank`, `world`: a later ring of the same job (the fault drill's)."""
        path = self.uid_path(tag)
        rank = self.rank if rank is None else rank
        world = self.world if world is None else world
        if rank == 0:
            uid = N.unique_id()
            tmp = f"{path}.{os.getpid()}.tmp"
            with open(tmp, "wb") as f:
                f.write(uid)
            os.replace(tmp, path)
        else:
            t0 = time.monotonic()
            while True:
                try:
                    if os.stat(path).st_mtime >= self.t_start - 120.0:
                        with open(path, "rb") as f:
                            uid = f.read()
                        if len(uid) == N.GOL_UNIQUE_ID_BYTES:
                            break
                except OSError:
                    pass
                if time.monotonic() - t0 > timeout:
                    raise SystemExit(f"rank {rank}: no RCCL id from rank 0 at {path} after {timeout:.0f} s (the file "
                                     "is keyed by MASTER_ADDR:MASTER_PORT and the launch: GOL_BENCH_RUN_ID if set, "
                                     "else the ranks' common parent process -- a launcher whose ranks have "
                                     "different parents must set GOL_BENCH_RUN_ID to one value on every rank)")
                time.sleep(0.01)
        eng.comm_init(uid, rank, world)
        if world > 1:
            eng.allreduce_u64([0])  # every rank has read the id
        if rank == 0:
            try:
                os.unlink(path)
            except OSError:
                pass
        if not tag:
            self.eng = eng

    def barrier(self):
        if self.world > 1:
            self.eng.allreduce_u64([0])

    def gather(self, row):
        """Every rank's `row` (equal-length u64 list): a world x len(row)
        table, rank r in row r (an all-reduce of one-hot rows)."""
        import numpy as np
        k = len(row)
        if self.world == 1:
            return [list(int(x) for x in row)]
        buf = np.zeros(self.world * k, dtype=np.uint64)
        buf[self.rank * k:(self.rank + 1) * k] = np.asarray(row, dtype=np.uint64)
        out = self.eng.allreduce_u64(buf)
        return [[int(x) for x in out[r * k:(r + 1) * k]] for r in range(self.world)]


def timed_run(eng, job, steps, warmup, with_hash):
    """W untimed + K timed generations.  Returns (seconds, kernel ms,
    launches, generations covered by them, probe clock GHz, hashes): hashes
    = the W + K per-generation partial hashes of this shard when with_hash.
    `job`: the Job whose ranks step together, or None (this GPU alone)."""
    ranks = job is not None and job.world > 1
    hw = eng.step(warmup, hashes=with_hash) if warmup > 0 else None
    eng.sync()
    eng.profile(True)
    eng.profile_reset()
    if ranks:
        job.barrier()
    eng.sync()
    t0 = time.perf_counter()
    ht = eng.step(steps, hashes=with_hash)
    eng.sync()
    # the clock stops when this rank's work is done; the closing barrier and
    # the max over ranks then give the job's time
    dt = time.perf_counter() - t0
    if ranks:
        job.barrier()
    kms, launches, gens = eng.profile_read()
    clock = eng.profile_clock()  # GHz the timed launches ran at (in-kernel probe)
    timed_run.stats = eng.profile_stats()
    eng.profile(False)
    if ranks:
        # every rank's own time (rank order) -> the job's time is their max
        timed_run.rank_times = [r[0] / 1e9 for r in job.gather([round(dt * 1e9)])]
        dt = max(timed_run.rank_times)
    hashes = None
    if with_hash:
        import numpy as np
        hashes = np.concatenate([h for h in (hw, ht) if h is not None]).astype(np.uint64)
    return dt, kms, launches, gens, clock, hashes


GOLDEN_SEED = 0x5EED


def golden_path(W, H):
    return os.path.join("tests", "golden", f"bench_{W}.json" if W == H else f"bench_{W}x{H}.json")


def golden_hashes(W, H):
    """Global state hashes of a bench board (W x H torus, B3/S23, seed
    0x5EED) at epochs 0, 1, ..., from tests/golden/bench_<W>[x<H>].json --
    written by tests/golden/make_bench_golden.py with the CPU oracle (a data
    file: bench never runs the oracle to check itself).  None if there is no
    table."""
    try:
        with open(os.path.join(ROOT, golden_path(W, H))) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("board") != [W, H] or d.get("seed") != GOLDEN_SEED or d.get("rule") != "B3/S23":
        return None
    return [int(x, 16) for x in d["hashes"]]


def global_hash(eng, job):
    """The whole board's state hash: gol_hash of every shard, summed over the
    ranks with gol_comm_allreduce_u64 (RCCL) -- the hash is a sum mod 2^64, so
    the N shards' partials add up to the N = 1 value."""
    import numpy as np
    h = np.array([eng.hash()], dtype=np.uint64)
    if job is not None and job.world > 1:
        h = eng.allreduce_u64(h)
    return int(h[0])


class Parity:
    """bench.py's self-check against the committed golden hashes: every board
    it times is checked at the epoch its window ends on (the shards of every
    rank through the summed hash at N > 1, so the multi-GPU line records
    whether the RCCL halo exchange kept the board bit-exact;
    CellActor.scala:71-77, NextStateCellGathererActor.scala:32-36 are the
    exchange it replaces).  Each check is also returned, for the sub-line it
    belongs to."""

    def __init__(self):
        self.tables = {}
        self.sources = {}  # shape -> the file a table came from, when not tests/golden/bench_*.json
        self.checks = []

    def add_table(self, shape, hashes, source):
        """A golden table (epoch k -> hash) from another committed file."""
        self.tables[shape] = list(hashes)
        self.sources[shape] = source

    def _golden(self, shape, epoch):
        if shape not in self.tables:
            self.tables[shape] = golden_hashes(*shape)
        g = self.tables[shape]
        return g[epoch] if g is not None and epoch < len(g) else None

    def board(self, what, shape, epoch, value):
        g = self._golden(shape, epoch)
        c = {"what": what, "board": f"{shape[0]}x{shape[1]}", "epoch": epoch, "hash": f"{value:#018x}",
             "golden": None if g is None else f"{g:#018x}", "match": None if g is None else value == g}
        self.checks.append(c)
        return {k: c[k] for k in ("epoch", "hash", "golden", "match")}

    def sequence(self, what, shape, first_epoch, values):
        gs = [self._golden(shape, first_epoch + k) for k in range(len(values))]
        known = [(first_epoch + k, int(v), g) for k, (v, g) in enumerate(zip(values, gs)) if g is not None]
        bad = [e for e, v, g in known if v != g]
        c = {"what": what, "board": f"{shape[0]}x{shape[1]}", "epochs": [first_epoch, first_epoch + len(values) - 1],
             "checked": len(known), "mismatched_epochs": bad[:16],
             "last_hash": f"{int(values[-1]):#018x}" if len(values) else None,
             "match": (not bad) if known else None}
        self.checks.append(c)
        return c

    def failed(self, allow_unchecked=False):
        """The checks that did not match (or, unless allow_unchecked, that had
        no golden value): short labels for the line's closing parity_failed."""
        return [f'{c["what"]} [{c["board"]}]: ' + ("mismatch" if c["match"] is False else "no golden value")
                for c in self.checks if c["match"] is False or (c["match"] is None and not allow_unchecked)]

    def report(self):
        ms = [c["match"] for c in self.checks]
        used = sorted(self.sources.get(k, golden_path(*k)) for k, v in self.tables.items() if v is not None)
        return {"golden": (", ".join(used) + " (CPU oracle, tests/golden/make_bench_golden.py; "
                           "parity unpinned: the reference ships no vectors)") if used else None,
                "checks": self.checks,
                "match": None if not ms or any(m is None for m in ms) else all(ms)}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_rate(O, width, H, threads, seconds):
    board = O.seed_packed(width, H, GOLDEN_SEED)
    O.run_packed(board, width, 1, nthreads=threads, want_hashes=False)  # warm
    gens, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        board, _ = O.run_packed(board, width, 4, nthreads=threads, want_hashes=False)
        gens += 4
    dt = time.perf_counter() - t0
    return width * H * gens / dt / 1e9, gens, dt


SCALAR_EDGE = 4096
# The reference's own ceiling: its default board is
# size (6, 6), i.e. the inclusive 7 x 7 = 49 cells (application.conf:31-33,
# BoardCreator.scala:47-53), and the frontend advances at most one generation
# per `tick` = 3000 ms (application.conf:40, BoardCreator.scala:105-116).
AKKA_CELLS, AKKA_TICK_S = 49, 3.0


def _scalar_rate(O, seconds):
    """The scalar per-cell oracle (oracle_step_cells, gol_oracle.c: the literal
    restatement of package.scala:17-28 + NextStateCellGathererActor.scala:39-46,
    one thread) on the 4096^2 torus from the golden seed, for at least one
    generation and about `seconds`; the board it ends on is checked against
    tests/golden/golden.json's per-generation hashes."""
    E = SCALAR_EDGE
    cells = O.unpack(O.seed_packed(E, E, GOLDEN_SEED), E)
    gens, t0 = 0, time.perf_counter()
    while gens == 0 or time.perf_counter() - t0 < seconds:
        cells = O.step_cells(cells, O.TORUS, O.LIFE)
        gens += 1
    dt = time.perf_counter() - t0
    h = O.hash_packed(O.pack(cells), E)
    golden = None
    try:
        with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
            for ent in json.load(f)["torus"]:
                if (ent["W"], ent["H"], ent["seed"], ent["rule"]) == (E, E, GOLDEN_SEED, "life") and gens <= ent["gens"]:
                    golden = int(ent["hashes"][gens - 1])
    except (OSError, ValueError, KeyError):
        pass
    return E * E * gens / dt / 1e9, gens, dt, {"epoch": gens, "hash": f"{h:#018x}",
                                              "golden": None if golden is None else f"{golden:#018x}",
                                              "match": None if golden is None else h == golden}


def cpu_baseline(width, seconds):
    """The CPU figures of SURVEY.md section 8(d), each on a bounded sample:

    * packed_port (the line's value): the oracle's bit-packed, bit-sliced,
      OpenMP step on a torus of the same width and 1024 rows, run for
      ~`seconds`, on the CPU share the harness grants the job
      (OMP_NUM_THREADS: 16 threads per GPU on the pool's boxes;
      sched_getaffinity when unset).  More threads than the job's cgroup
      quota would only time-slice on the same CPUs, so no such figure is
      reported;
    * scalar_4096: the scalar per-cell oracle, one thread, on configs[1]'s
      4096^2 torus (about `seconds`), its end state checked against the
      golden hashes;
    * akka_derived_ceiling: the reference's own rate bound, derived (not
      measured: no JVM on the box) from its default board and tick."""
    from oracle import oracle as O
    affinity = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(share, affinity) if share > 0 else affinity
    quota = cgroup_cpus()
    if quota:
        threads = max(1, min(threads, int(quota)))
    H = 1024
    v, gens, dt = _cpu_rate(O, width, H, threads, seconds)
    out = {"value": round(v, 3), "unit": "GCUPS", "cores": threads,
           "kind": "port", "nproc": os.cpu_count(), "affinity": affinity, "cpu_model": cpu_model(),
           "threads_source": "OMP_NUM_THREADS (the job's CPU share)" if share > 0 else "sched_getaffinity",
           "sample": f"oracle_run_packed (oracle/gol_oracle.c, bit-sliced, OpenMP), {width}x{H} torus B3/S23 "
                     f"slice of the same workload, {gens} generations in {dt:.1f} s on {threads} threads"}
    if quota:
        out["cgroup_cpu_quota"] = quota
    out["packed_port"] = {k: out[k] for k in ("value", "unit", "cores", "kind", "sample")}
    out["packed_port"]["model"] = "bit-packed 32 cells per word, bit-sliced adder, OpenMP over rows"
    vs, gs, dts, par = _scalar_rate(O, seconds)
    out["scalar_4096"] = {"value": round(vs, 5), "unit": "GCUPS", "cores": 1, "kind": "port",
                          "model": "scalar per-cell oracle (oracle_step_cells): 8 wrapped neighbour reads and a "
                                   "rule lookup per cell, the reference's per-cell algorithm restated",
                          "sample": f"{SCALAR_EDGE}x{SCALAR_EDGE} torus B3/S23 (BASELINE.json configs[1]) from seed "
                                    f"0x5EED, {gs} generations in {dts:.1f} s on 1 thread",
                          "parity": par}
    out["akka_derived_ceiling"] = {
        "value": AKKA_CELLS / AKKA_TICK_S / 1e9, "unit": "GCUPS", "cores": None, "kind": "derived",
        "cell_updates_per_s": round(AKKA_CELLS / AKKA_TICK_S, 3),
        "sample": "not measured (no JVM on the box): the reference's default 7 x 7 board (size (6, 6), "
                  "application.conf:31-33) advances at most one generation per 3000 ms tick "
                  "(application.conf:40, BoardCreator.scala:105-116) = 49 / 3 cell updates per second"}
    return out


def cgroup_cpus():
    """CPUs the job's cgroup (v2 cpu.max, else v1 cfs quota) allows, or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return None if q == "max" else int(q) / int(p)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            p = int(f.read())
        return None if q <= 0 else q / p
    except (OSError, ValueError):
        return None


def pmc_launch():
    """profiles/pmc_launch.json (scripts/gpu_pmc.sh + scripts/pmc_launch.py):
    per-launch PMC numbers keyed 'WxH/mode/G<g>/h<hash>'."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_launch.json")) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def plan_pmc(shape, mode, plan, hashed):
    """PMC numbers of a pass plan's launches: mean HBM bytes per launch,
    time-weighted clock, cell-weighted VALU per word-generation.  None if a
    depth of the plan was not profiled."""
    table = pmc_launch()
    ents = [table.get(f"{shape}/{mode}/G{g}/h{int(hashed)}") for g in plan]
    if not ents or any(e is None for e in ents):
        return None
    t = sum(e["launch_ms"] for e in ents)
    return {"hbm_bytes": sum(e["hbm_bytes"] for e in ents) / len(ents),
            "clock_ghz": sum(e["clock_ghz"] * e["launch_ms"] for e in ents) / t,
            "valu_per_word_gen": sum(e["valu_per_word_gen"] * e["generations_per_launch"] for e in ents) /
            sum(e["generations_per_launch"] for e in ents),
            "keys": sorted({f"{shape}/{mode}/G{g}/h{int(hashed)}" for g in plan})}


def valu_peak_gcups(mix, clock_ghz):
    cycles = sum(n * c for n, c in mix.values())
    return SIMDS * clock_ghz * 1e9 / cycles * CELLS_PER_WAVE_INSTR / 1e9, cycles


def guide_peak_gcups(valu_per_word_gen, clock_ghz=CLOCK_MAX_GHZ):
    """VALU-issue ceiling at the guide's 2 cycles per wave64 instruction:
    every SIMD issuing one instruction per 2 cycles at `clock_ghz`, each
    instruction one word (32 cells) on each of 64 lanes."""
    return SIMDS * clock_ghz * 1e9 / (valu_per_word_gen * GUIDE_CYCLES_PER_VALU) * CELLS_PER_WAVE_INSTR / 1e9


def issue_rate(gcups, valu_per_word_gen, clock_ghz):
    """Wave-VALU instructions issued per cycle per SIMD by launches running
    at `gcups` with `valu_per_word_gen` instructions per word-generation at
    `clock_ghz` (0.5 = the guide's issue ceiling)."""
    return gcups * 1e9 / CELLS_PER_WAVE_INSTR * valu_per_word_gen / (SIMDS * clock_ghz * 1e9)


def copy_peak():
    """The measured stream-copy peak (read + write GB/s): profiles/copy_peak.json,
    written from scripts/micro/copy_bw.hip's last line on an MI355X box.
    None if absent."""
    try:
        with open(os.path.join(ROOT, COPY_PEAK_FILE)) as f:
            d = json.load(f)
        return {"gbs": float(d["copy_peak_gbs"]), "variant": d.get("variant"),
                "source": f"{COPY_PEAK_FILE} ({d.get('measured', 'scripts/micro/copy_bw.hip')})"}
    except (OSError, ValueError, KeyError):
        return None


def compact_plan(plan):
    """A long pass plan as "n x G" runs, e.g. "128 x 8" or "7 x 12 + 2 x 9"."""
    runs = []
    for g in plan:
        if runs and runs[-1][1] == g:
            runs[-1][0] += 1
        else:
            runs.append([1, g])
    return " + ".join(f"{n} x {g}" for n, g in runs)


def roofline(kms, launches, gens_covered, cells, plan, shape, mode, hashed=False, clock=None):
    """Roofline of the dominant kernel (see the module docstring).  `clock`:
    GHz the timed launches held, from the in-kernel probe (gol_profile_clock):
    it prices the held_clock diagnostic, never the primary frac."""
    if not launches:
        return None
    avg_s = kms / 1e3 / launches
    gpl = gens_covered / launches
    gcups = cells * gpl / avg_s / 1e9
    algo = cells * gpl * BYTES_PER_CELL_UPDATE
    common = {"avg_launch_ms": round(avg_s * 1e3, 4), "launches": launches, "generations_per_launch": gpl,
              "pass_plan": plan if len(plan) <= 16 else compact_plan(plan)}
    pmc = plan_pmc(shape, mode, plan, hashed)
    if set(plan) == {1}:  # single-generation passes: a stream over the plane, HBM-bound
        r = {"bound": "hbm", "achieved": round(algo / avg_s / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(algo / avg_s / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
             "algorithmic_bytes_per_launch": algo, **common}
        cp = copy_peak()
        if cp:
            r["copy_peak"] = cp
            r["frac_of_copy_peak"] = round(algo / avg_s / 1e9 / cp["gbs"], 4)
        if pmc:
            r["traffic"] = round(pmc["hbm_bytes"])
            r["measured_hbm_gbs"] = round(pmc["hbm_bytes"] / avg_s / 1e9, 1)
            r["measured_hbm_frac"] = round(pmc["hbm_bytes"] / avg_s / 1e9 / HBM_PEAK_GBS, 4)
            r["traffic_source"] = ("profiles/pmc_launch.json " + ", ".join(pmc["keys"]) +
                                   " (rocprofv3 PMC passes of the same kernels; not measured in this run)")
        return r
    mix = VALU_MIX_HASH if hashed else VALU_MIX
    # frac: against the VALU-issue ceiling at the guide's max clock (2.4 GHz,
    # MI355X_MICROARCH.md) -- the peak the chip is specified for.  The clock
    # these launches actually held (in-kernel probe, gol_profile_clock) only
    # prices the separate issue-efficiency diagnostic under held_clock.
    peak_max, cycles = valu_peak_gcups(mix, CLOCK_MAX_GHZ)
    n_valu = sum(n for n, _ in mix.values())
    peak_guide = guide_peak_gcups(n_valu)
    r = {"bound": "valu", "achieved": round(gcups, 1), "peak": round(peak_max, 1), "unit": "GCUPS",
         "frac": round(gcups / peak_max, 4), "frac_kind": "mix-priced: the loop's instruction mix at the measured "
                                                          "per-op issue costs (profiles/r01_valu_op_costs.txt)",
         "frac_guide_issue": round(gcups / peak_guide, 4),
         "peak_guide_issue": round(peak_guide, 1),
         "guide_issue_note": f"{n_valu:g} VALU per word-generation at the guide's {GUIDE_CYCLES_PER_VALU:g} cycles "
                             "per wave64 instruction (MI355X_MICROARCH.md), 2.4 GHz",
         "traffic": round(pmc["hbm_bytes"]) if pmc else None,
         "traffic_source": ("profiles/pmc_launch.json " + ", ".join(pmc["keys"]) +
                            " (rocprofv3 PMC passes of the same kernels; not measured in this run)") if pmc else None,
         "peak_clock_ghz": CLOCK_MAX_GHZ,
         "valu": {"instructions_per_word_generation": {k: n for k, (n, _) in mix.items()},
                  "cycles_per_word_generation": round(cycles, 2),
                  "measured_valu_per_word_generation": round(pmc["valu_per_word_gen"], 2) if pmc else None,
                  "circuit": "row-pair-shared B3/S23 (pair_sum + rule_b3s23_pair)",
                  "source": "loop census scripts/isa_loop.py; issue costs profiles/r01_valu_op_costs.txt"},
         **common}
    held = {"clock_pmc_ghz": round(pmc["clock_ghz"], 3) if pmc else None}
    vpwg = pmc["valu_per_word_gen"] if pmc else n_valu
    clk_issue = clock or (pmc["clock_ghz"] if pmc else None)
    if clk_issue:
        r["issue_rate"] = {"wave_valu_per_cycle_per_simd": round(issue_rate(gcups, vpwg, clk_issue), 4),
                           "guide_max": round(1 / GUIDE_CYCLES_PER_VALU, 4), "clock_ghz": round(clk_issue, 3),
                           "valu_per_word_generation": round(vpwg, 3),
                           "source": ("PMC VALU per word-generation" if pmc else "loop census") + " at the " +
                                     ("in-kernel probe clock" if clock else "PMC clock")}
    cp = copy_peak()
    if cp:
        r["copy_peak"] = cp
    if clock:
        peak_held, _ = valu_peak_gcups(mix, clock)
        held.update({"ghz": round(clock, 3), "peak_at_held_clock": round(peak_held, 1),
                     "issue_efficiency": round(gcups / peak_held, 4),
                     # the rate per held GHz: flat across boxes whose power limit holds
                     # different clocks (profiles/r06_size_scan.txt)
                     "gcups_per_ghz": round(gcups / clock, 1),
                     "source": "in-kernel probe of these timed launches: every sampled workgroup's core-clock "
                               "(s_memtime) and 100 MHz reference (s_memrealtime) ticks, summed (gol_profile_clock)"})
    r["held_clock"] = held
    if pmc:
        gbs = pmc["hbm_bytes"] / avg_s / 1e9
        r["hbm"] = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(gbs / HBM_PEAK_GBS, 4),
                    "note": "physical HBM traffic per launch (PMC FETCH_SIZE x2 + WRITE_SIZE) / launch time",
                    "traffic_source": "profiles/pmc_launch.json " + ", ".join(pmc["keys"])}
    r["hbm_effective"] = {"achieved": round(algo / avg_s / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(algo / avg_s / 1e9 / HBM_PEAK_GBS, 4),
                          "algorithmic_bytes_per_launch": algo,
                          "note": "0.25 B per cell-update (SURVEY.md 8d) x generations fused per launch: "
                                  "exceeds 1 by temporal blocking, not a bandwidth"}
    return r


def kernel_label(info, depths, ilv=2):
    """Name of the kernel instances the timed passes launch (depths: the pass
    plan, gol_pass_plan): the strip width (gol_occupancy) gives the words per
    lane; multi-generation passes at 8-byte lanes or narrower run the
    horizontal-first kernel (gol_stencil.h launch_one); ilv = the board's
    interleave (gol_device_layout)."""
    gs = sorted(set(depths)) or [1]
    waves, strip = info.get(gs[-1], (0, 0))
    lay = {1: "row-major", 2: "pairs"}.get(ilv, ilv)
    if gs == [1]:
        vec = strip // 64 if strip else "VEC"
        return f"gol::dev::step_kernel<{vec},LIFE,{lay}>"
    vec = strip // 62 if strip else 0
    name = "multistep_hg_kernel" if vec in (1, 2) else "multistep_kernel"
    return f"gol::dev::{name}<{vec or 'VEC'},{'|'.join(map(str, gs))},LIFE,{lay}> ({waves} waves/CU resident)"


def settle(eng, ms, chunk, job=None):
    """Step `eng` untimed until `ms` of wall time has passed: after an idle
    gap (context creation, seeding, a 16 GiB allocation) the chip's clock
    dips and recovers over ~20 launches (profiles/r02_warmup_curve.txt),
    longer than a short window.  With ranks, rank 0's clock decides when all
    stop (every rank must step the same generations: the passes exchange
    halos)."""
    ranks = job is not None and job.world > 1
    t0 = time.perf_counter()
    while True:
        eng.step(chunk)
        eng.sync()
        go = int((time.perf_counter() - t0) * 1e3 < ms)
        if ranks:
            go = int(eng.allreduce_u64([go if job.rank == 0 else 0])[0])
        if not go:
            return


def fresh_window(eng, job, steps, warmup, with_hash, settle_ms, chunk):
    """The bench's window on a board: seed, settle (untimed), re-seed, then
    W warm-up and K timed generations -- so the window ends at epoch W + K
    from the seed whatever the settle did, and its hash has a golden value."""
    if settle_ms > 0:
        eng.seed(GOLDEN_SEED)
        settle(eng, settle_ms, chunk, job)
    eng.seed(GOLDEN_SEED)
    return timed_run(eng, job, steps, warmup, with_hash)


def secondary_run(GolEngine, a, local, parity=None):
    """BASELINE.json configs[2]: the 65536^2 single-GPU roofline run.

    Three windows on the same board, each from the seed, each checked
    against tests/golden/bench_65536.json at the epoch it ends on: SURVEY.md
    section 8(d)'s minimum (>= 10 warm-up, >= 100 timed generations: 4 ms at
    65536^2, inside the clock's recovery after the idle gap) as
    "short_window"; the reported value over >= 1024 generations after a 50 ms
    settle; and the same board one generation per HBM pass (the pure
    bandwidth case, north_star: >= 70 % of peak HBM at 65536^2).
    `parity`: where the checks go (None: not recorded)."""
    S = 65536
    shape = (S, S)
    chk = parity.board if parity is not None else (lambda *x: None)
    out = {"workload": "65536x65536 torus B3/S23 on 1 GPU (BASELINE.json configs[2])"}
    with GolEngine(S, S, topology="torus", rule="life", device=local) as e2:
        e2.set_tuning(band_rows=a.band, gens_per_pass=a.gpp)
        n_s, w_s = max(a.steps, 102), max(a.warmup, 12)
        dt_s, _, _, _, _, _ = fresh_window(e2, None, n_s, w_s, a.hash, 0, 0)
        p_s = chk("65536^2 short window: gol_hash after W + K", shape, n_s + w_s, e2.hash())
        n2 = max(a.steps, 1024)
        dt2, kms2, l2, g2, c2, _ = fresh_window(e2, None, n2, 0, a.hash, 50.0, 64)
        p2 = chk("65536^2 window: gol_hash after K", shape, n2, e2.hash())
        plan2 = e2.pass_plan(min(n2, 1024), hashes=a.hash)
        e2.set_tuning(band_rows=a.band, gens_per_pass=1)
        n1 = max(a.steps, 256)
        dt1, kms1, l1, g1, c1, _ = fresh_window(e2, None, n1, 0, a.hash, 50.0, 16)
        p1 = chk("65536^2 single-generation passes: gol_hash after K", shape, n1, e2.hash())
    sh = f"{S}x{S}"
    r2 = roofline(kms2, l2, g2, S * S, plan2, sh, "N1", a.hash, c2)
    r1 = roofline(kms1, l1, g1, S * S, [1] * n1, sh, "N1", a.hash, c1)
    out.update({
        "value": round(S * S * n2 / dt2 / 1e9, 2), "unit": "GCUPS", "steps": n2,
        "warmup": "50 ms settled, re-seeded", "ms_per_step": round(dt2 / n2 * 1e3, 4), "roofline": r2,
        "parity": p2,
        "short_window": {"value": round(S * S * n_s / dt_s / 1e9, 2), "unit": "GCUPS", "steps": n_s,
                         "warmup": w_s, "ms_per_step": round(dt_s / n_s * 1e3, 4), "parity": p_s,
                         "note": "fresh seed right after context creation: inside the clock's recovery"},
        "single_generation_passes": {"value": round(S * S * n1 / dt1 / 1e9, 2), "unit": "GCUPS", "steps": n1,
                                     "warmup": "50 ms settled, re-seeded", "ms_per_step": round(dt1 / n1 * 1e3, 4),
                                     "roofline": r1, "parity": p1,
                                     # the same bytes over the wall-clock time per generation
                                     # (launch gaps included), beside the kernel-time frac
                                     "hbm_frac_from_ms_per_step": round(
                                         S * S * BYTES_PER_CELL_UPDATE / (dt1 / n1) / 1e9 / HBM_PEAK_GBS, 4)}})
    return out


SMALL_EDGE, SMALL_GENS = 4096, 1000


def golden_small():
    """tests/golden/golden.json's 4096^2 torus (seed 0x5EED, B3/S23): the
    hashes at epochs 0..1000, or None."""
    try:
        with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
            for ent in json.load(f)["torus"]:
                if (ent["W"], ent["H"], ent["seed"], ent["rule"]) == (SMALL_EDGE, SMALL_EDGE, GOLDEN_SEED, "life"):
                    return [int(ent["hash0"])] + [int(h) for h in ent["hashes"]]
    except (OSError, ValueError, KeyError):
        pass
    return None


def small_board_run(GolEngine, local, parity):
    """BASELINE.json configs[1]: the 4096^2 torus for 1000 generations (2 MiB
    per plane: the board lives in the caches, so the pass is bound by the
    latency of each wave's row stream, not by HBM -- gol_schedule.cpp
    small_board_band).  One untimed run from the seed (code-object and clock
    warm-up), then timed from the seed again: unhashed, then with every
    generation's hash, each checked against tests/golden/golden.json."""
    S, n = SMALL_EDGE, SMALL_GENS
    shape = (S, S)
    g = golden_small()
    if g is not None and parity is not None:
        parity.add_table(shape, g, "tests/golden/golden.json (torus 4096^2, seed 0x5EED)")
    out = {"workload": f"{S}x{S} torus B3/S23, {n} generations from the seed (BASELINE.json configs[1])"}
    with GolEngine(S, S, topology="torus", rule="life", device=local) as e:
        for hashed in (False, True):
            e.seed(GOLDEN_SEED)
            e.step(n, hashes=hashed)
            e.sync()
            # kernel time: a profiled run (events around every launch)
            e.seed(GOLDEN_SEED)
            e.sync()
            e.profile(True)
            e.profile_reset()
            e.step(n, hashes=hashed)
            e.sync()
            kms, launches, _ = e.profile_read()
            e.profile(False)
            # wall time: the same run without the profiling events
            e.seed(GOLDEN_SEED)
            e.sync()
            t0 = time.perf_counter()
            hs = e.step(n, hashes=hashed)
            e.sync()
            dt = time.perf_counter() - t0
            rec = {"value": round(S * S * n / dt / 1e9, 1), "unit": "GCUPS", "wall_ms": round(dt * 1e3, 3),
                   "kernel_ms": round(kms, 3), "kernel_ms_source": "a separate profiled run of the same generations",
                   "launches": launches, "pass_plan": compact_plan(e.pass_plan(n, hashed))}
            if parity is not None:
                rec["parity"] = parity.board(f"configs[1] 4096^2 x {n}{' hashed' if hashed else ''}: gol_hash after "
                                             f"{n}", shape, n, e.hash())
                if hashed:
                    seq = parity.sequence(f"configs[1] 4096^2: the {n} fused per-generation hashes", shape, 1, hs)
                    rec["parity_per_generation"] = {k: seq[k] for k in ("checked", "mismatched_epochs", "match")}
            out["with_state_hash" if hashed else "unhashed"] = rec
    out["value"] = out["unhashed"]["value"]
    out["unit"] = "GCUPS"
    return out


AKKA_DEFAULT_SEED = 42  # tests/golden/golden.json ref_default entry (java.util.Random seed)


def default_board_run(GolEngine, local, parity):
    """BASELINE.json configs[0] on this engine: the reference's own default
    board -- size (6, 6), i.e. 7 x 7 cells with neighbours clipped to
    [0, 6) x [0, 6) (application.conf:31-33, package.scala:17-28) -- from the
    java.util.Random(42) board of BoardCreator.scala:23 (the golden vectors'
    initial cells, a data file), 100 generations of the rule the reference
    actually runs (ref-effective: the identity) and of B3/S23.  Timed as the
    reference drives it -- one gol_step(1) per NextStep tick
    (BoardCreator.scala:113-116) -- and as one call; every generation's hash
    against golden.json.  The Akka cluster itself cannot run here (no JVM):
    its ceiling is one generation per 3000 ms tick (cpu_baseline)."""
    import numpy as np
    from gameoflife import codec
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        ent = next(e for e in json.load(f)["ref_default"] if e["java_seed"] == AKKA_DEFAULT_SEED)
    x, y = ent["w"], ent["h"]
    cells = np.array([[int(c) for c in r] for r in ent["initial"]], dtype=np.uint8)
    out = {"workload": f"the reference's default board: size ({x}, {y}) = {x + 1}x{y + 1} cells, ref-clipped, "
                       f"java.util.Random({AKKA_DEFAULT_SEED}) initial board, 100 generations (BASELINE.json configs[0])"}
    for rule in ("ref-effective", "life"):
        want = [int(h) for h in ent["modes"][rule]["hashes"]]
        n = len(want)
        with GolEngine(x + 1, y + 1, topology="ref-clipped", rule=rule, device=local) as e:
            e.load(codec.pack(cells))
            e.step(n)  # code-object / first-call warm-up
            res = {}
            for mode in ("per_tick", "one_call"):
                e.load(codec.pack(cells))
                e.sync()
                t0 = time.perf_counter()
                if mode == "per_tick":
                    hs = np.concatenate([e.step(1, hashes=True) for _ in range(n)])
                else:
                    hs = e.step(n, hashes=True)
                e.sync()
                dt = time.perf_counter() - t0
                ok = [int(h) for h in hs] == want
                if parity is not None:
                    parity.checks.append({"what": f"configs[0] default board, {rule}, {mode}: the {n} per-generation "
                                                  "hashes", "board": f"{x + 1}x{y + 1}", "epochs": [1, n],
                                          "checked": n, "match": ok})
                res[mode] = {"us_per_generation": round(dt / n * 1e6, 2),
                             "generations_per_s": round(n / dt), "parity": ok,
                             "vs_akka_tick": round(AKKA_TICK_S / (dt / n)),
                             }
            out[rule] = res
    out["note"] = ("vs_akka_tick: the reference's 3000 ms per generation (application.conf:40) over this engine's time "
                   "per generation on the same board; the Akka run itself is not measurable here (no JVM)")
    return out


def ring_stats(st, passes):
    """The self-ring windows' exchange figures (gol_profile_stats_read)."""
    n = max(st["exchanges"], 1)
    return {"exchange_ms_per_pass": round(st["exchange_ms"] / n, 4),
            "exchange_exposed_ms_per_pass": round(st["exchange_exposed_ms"] / n, 4),
            "boundary_ms_per_pass": round(st["boundary_ms"] / max(st["boundary_launches"], 1), 4),
            "pass_tail_ms_per_pass": round(st["pass_tail_ms"] / max(st["boundary_launches"], 1), 4),
            "halo_bytes_per_pass": round((st["halo_bytes_sent"] + st["halo_bytes_received"]) / max(passes, 1)),
            "passes": passes}


def ring_schedule_runs(GolEngine, N, a, local, eng, W, H, parity):
    """N = 1 only: the row-sharded (RCCL ring) schedule on this GPU, as a 1-rank
    self-ring (gol_ring.cpp one_pass: interior launch || G-row halo
    ncclSend/ncclRecv to itself, then the boundary rows on the edge stream).
    (1) the whole board, (2) one rank's shard of the N = 8 decomposition
    (262144 x 32768): what each of 8 ranks computes, without the xGMI latency
    of a real ring.  Every window starts from the seed and is checked against
    its golden table (bench_262144.json, bench_262144x32768.json)."""
    out = {}
    warm = "settled, re-seeded"
    eng.comm_init(N.unique_id(), 0, 1)
    dt, kms, launches, gcov, _, _ = fresh_window(eng, None, a.steps, a.warmup, False, 100.0, 12)
    st = timed_run.stats
    out["whole_board_self_ring"] = {
        "value": round(W * H * a.steps / dt / 1e9, 2), "unit": "GCUPS", "warmup": f"{a.warmup} ({warm})",
        "ms_per_step": round(dt / a.steps * 1e3, 4), "pass_plan": eng.pass_plan(min(a.steps, 1024)),
        "exchange": ring_stats(st, launches),
        "parity": parity.board("whole-board self-ring: gol_hash after W + K", (W, H), a.warmup + a.steps, eng.hash())}
    rows8 = H // 8
    shape8 = (W, rows8)
    with GolEngine(W, H, topology="torus", rule="life", device=local, row0=0, rows=rows8) as e8:
        e8.comm_init(N.unique_id(), 0, 1)  # a 1-rank ring over a shard-sized torus
        # First as an N = 8 rank meets the driver's window (main(), N > 1):
        # the GPU idle while the ranks initialise RCCL, the 65536^2 run, then
        # the rank's own settle, seed, W warm-up and K timed steps.
        time.sleep(1.0)
        if not a.no_secondary:
            secondary_run(GolEngine, a, local)
        dtf, _, _, _, _, _ = fresh_window(e8, None, a.steps, a.warmup, False, 100.0, 12)
        out["per_rank_shard_driver_window"] = {
            "shard": f"{W}x{rows8} (one rank of N = 8)", "value": round(W * rows8 * a.steps / dtf / 1e9, 2),
            "unit": "GCUPS", "warmup": f"{a.warmup} ({warm})", "ms_per_step": round(dtf / a.steps * 1e3, 4),
            "parity": parity.board("N = 8 rank's shard, driver's sequence: gol_hash after W + K", shape8,
                                   a.warmup + a.steps, e8.hash()),
            "note": "an N = 8 rank's sequence on this GPU (1 s idle for the communicator setup, the 65536^2 run, "
                    "the same settle and re-seed as main(), W warm-up and K timed steps); x 8 / the N = 1 value "
                    "is the per-cell efficiency that run can reach before any xGMI cost"}
        time.sleep(1.0)
        dt8, kms8, l8, g8, c8, _ = fresh_window(e8, None, a.steps, a.warmup, False, 100.0, 12)
        st8 = timed_run.stats
        p8 = parity.board("N = 8 rank's shard, self-ring: gol_hash after W + K", shape8, a.warmup + a.steps,
                          e8.hash())
        plan8 = e8.pass_plan(min(a.steps, 1024))
    out["per_rank_shard_self_ring"] = {
        "shard": f"{W}x{rows8} (one rank of N = 8)", "value": round(W * rows8 * a.steps / dt8 / 1e9, 2),
        "unit": "GCUPS", "warmup": f"{a.warmup} ({warm}, after 1 s idle)", "ms_per_step": round(dt8 / a.steps * 1e3, 4),
        "pass_plan": plan8, "exchange": ring_stats(st8, l8), "parity": p8,
        "interior_launch": roofline(kms8, l8, g8, W * max(rows8 - round(2 * g8 / max(l8, 1)), 0), plan8,
                                    f"{W}x{rows8}", "ring", False, c8)}
    return out


def N_layout(width):
    """Words per interleave group of a torus of `width` columns
    (gol_device_layout)."""
    from gameoflife import _native as N
    return N.device_layout(width)


def lib_fingerprint(info):
    """64-bit digest of the HIP and RCCL library paths (rank comparison)."""
    d = hashlib.sha1((info["hip_library"] + "|" + info["rccl_library"]).encode()).digest()
    return int.from_bytes(d[:8], "little")


def rank_table(job, N, stats, dt, info):
    """Every rank's diagnostics at N > 1, gathered over
    RCCL: its window time, its interior launches, the halo exchange on its
    comm stream, its boundary launches, halo bytes, the runtime it ran on and
    the HIP statuses RCCL left behind in it."""
    absorbed, _ = N.absorbed()
    row = [round(dt * 1e9), round(stats["kernel_ms"] * 1e6), stats["launches"], round(stats["exchange_ms"] * 1e6),
           stats["exchanges"], round(stats["boundary_ms"] * 1e6), stats["boundary_launches"],
           stats["halo_bytes_sent"], stats["halo_bytes_received"], absorbed, info["hip_runtime_version"],
           info["rccl_version"], lib_fingerprint(info), round(stats["exchange_exposed_ms"] * 1e6),
           round(stats["pass_tail_ms"] * 1e6)]
    return job.gather(row)


def drill_error_files(job):
    """The files in which ranks whose fault drill raised left their exception
    (fault_drill), for rank 0's watchdog."""
    import glob
    return sorted(glob.glob(glob.escape(job.uid_path("fault_error")) + ".r*"))


def drill_errors(job):
    """{rank: exception text} from drill_error_files."""
    out = {}
    for p in drill_error_files(job):
        try:
            with open(p) as f:
                out[p.rsplit(".r", 1)[1]] = f.read()
        except OSError:
            pass
    return out


def fault_drill(job, N, GolEngine, eng, a, W, H, local, parity):
    """BASELINE.json configs[4] at N > 1, after the timed windows: the ranks
    lose rank min(3, N - 1) after generation 25 of 50 (checkpoints every 10)
    and re-spawn its shard on the rank above it, which replays it alone from
    its checkpoint and the light cone; the N - 1 survivors rebuild the RCCL
    ring and step on to 50 (gameoflife.elastic.ring_fault_drill; the
    reference's re-deploy of a dead cell, BoardCreator.scala:120-154).  Every
    global hash is checked against bench_262144.json.  Returns (the sub-line
    or None off rank 0, this rank's context afterwards -- None on the lost
    rank)."""
    import shutil
    import numpy as np
    from gameoflife.elastic import ring_fault_drill
    # The checkpoint files: every rank's shard, two epochs at the peak (a new
    # file is written before the previous one is removed) -- twice the board.
    # The first candidate directory with room for them (the same list on
    # every rank of the node); rank 0's choice is all-reduced so all agree.
    need = 2 * W * H // 8 + (1 << 30)
    cands = [d for d in (os.environ.get("GOL_BENCH_CKPT_DIR"), tempfile.gettempdir(), "/dev/shm") if d]
    pick = 0
    if job.rank == 0:
        for k, d in enumerate(cands):
            try:
                if shutil.disk_usage(d).free >= need:
                    pick = k + 1
                    break
            except OSError:
                pass
    pick = int(eng.allreduce_u64(np.array([pick], dtype=np.uint64))[0])
    if pick == 0:
        return ({"status": "skipped", "reason": f"no directory among {cands} has {need / 2**30:.0f} GiB free "
                 "for the checkpoint files"} if job.rank == 0 else None), eng
    ckpt = os.path.join(cands[pick - 1], os.path.basename(job.uid_path("fault_ckpt")) + "_dir")
    if job.rank == 0:
        shutil.rmtree(ckpt, ignore_errors=True)
        os.makedirs(ckpt)
        for p in drill_error_files(job):  # a crashed earlier launch's reports
            os.unlink(p)
    job.barrier()
    make = lambda r0, n: GolEngine(W, H, topology="torus", rule="life", device=local, row0=r0, rows=n)  # noqa: E731
    join = lambda e, tag, r, w: job.join(e, N, tag=tag, rank=r, world=w)  # noqa: E731
    t0 = time.perf_counter()
    try:
        eng, rep = ring_fault_drill(eng, make, join, job.rank, job.world, W, H, ckpt, seed=GOLDEN_SEED, victim=3,
                                    kill_at=25, gens=50, every=10)
    except Exception as exc:  # noqa: BLE001 -- reported on the line; peers left in a collective meet the watchdog
        parity.checks.append({"what": "fault drill", "board": f"{W}x{H}", "error": repr(exc), "match": False})
        print(f"bench.py rank {job.rank}: fault drill failed: {exc!r}", file=sys.stderr, flush=True)
        # for rank 0's watchdog: its peers are now stuck in a collective this
        # rank will never join, and the line should say why
        try:
            with open(f"{job.uid_path('fault_error')}.r{job.rank}", "w") as f:
                f.write(repr(exc)[:2000])
        except OSError:
            pass
        if job.rank != 0:
            return None, None
        shutil.rmtree(ckpt, ignore_errors=True)
        rec = {"status": "error", "error": repr(exc)}
        errs = {r: e for r, e in drill_errors(job).items() if r != "0"}
        if errs:  # a peer raised first (rank 0's own error is then the broken collective)
            rec["rank_errors"] = errs
            parity.checks.append({"what": "fault drill (peers)", "board": f"{W}x{H}", "error": repr(errs),
                                  "match": False})
        return rec, None
    if eng is None:  # the lost rank: its context is gone, it sits out the rest
        return None, None
    nw, nr = rep["world_after"], job.rank if job.rank < rep["victim_rank"] else job.rank - 1

    def ring_max(x):
        row = np.zeros(nw, dtype=np.uint64)
        row[nr] = round(x * 1e9)
        return float(eng.allreduce_u64(row).max()) / 1e9 if nw > 1 else x

    rec, aft, ck = ring_max(rep["recovery_s"]), ring_max(rep["after_s"]), ring_max(rep["checkpoint_s"])
    wall = ring_max(time.perf_counter() - t0)
    shape, c, k = (W, H), rep["checkpoint_epoch"], rep["kill_at"]
    checks = [
        parity.sequence("fault drill: global hashes before the loss (every rank)", shape, 1, rep["before"]),
        parity.sequence("fault drill: the replayed block's partials + the survivors' (epochs after the checkpoint)",
                        shape, c + 1, rep["replayed"]),
        {**parity.board("fault drill: gol_hash over the rebuilt ring at the loss epoch", shape, k,
                        rep["at_recovery"]), "what": "at recovery"},
        parity.sequence("fault drill: fused hashes on the rebuilt ring", shape, k + 1, rep["after"]),
        {**parity.board("fault drill: gol_hash at the end", shape, rep["generations"], rep["final"]), "what": "final"},
    ]
    if job.rank == 0:
        shutil.rmtree(ckpt, ignore_errors=True)  # every survivor has read what it needed
    if job.rank != 0:
        return None, eng
    after_gens = rep["generations"] - k
    ms = [c_.get("match") for c_ in checks]
    return {
        "status": "ok",
        "workload": f"{W}x{H} torus B3/S23 over {job.world} ranks: rank {rep['victim_rank']} lost after generation "
                    f"{k} of {rep['generations']} (BASELINE.json configs[4]), its shard re-spawned on rank "
                    f"{rep['host_rank']}'s GPU, {nw} ranks after",
        "checkpoint_every": rep["checkpoint_every"], "checkpoint_epoch": c,
        "replayed_generations": rep["replayed_generations"], "world_after": nw,
        "checkpoint_s_max": round(ck, 3),
        "recovery_ms": round(rec * 1e3, 1),
        "after": {"generations": after_gens, "ms_per_step": round(aft / max(after_gens, 1) * 1e3, 4),
                  "value": round(W * H * after_gens / aft / 1e9, 2) if aft > 0 else None, "unit": "GCUPS",
                  "note": "fused per-generation hashes on the N - 1 ring, one rank holding two shards"},
        "wall_s": round(wall, 3),
        "parity": {"match": None if any(m is None for m in ms) else all(ms),
                   "checks": [{kk: c_[kk] for kk in ("epochs", "epoch", "checked", "mismatched_epochs", "match")
                               if kk in c_} for c_ in checks]},
        "note": "recovery_ms: loss -> the host replayed the lost block (gol_replay from its checkpoint and the "
                "light cone read back from the checkpoint files) and merged it, and the survivors joined the "
                "new RCCL ring (max over the survivors)",
    }, eng


def main():
    a = parse()
    # one JSON line on stdout: native libraries (RCCL's version banner at
    # communicator creation) write to fd 1, so it points at stderr until the
    # result is printed on the saved descriptor
    sys.stdout.flush()
    result_fd = os.dup(1)
    os.dup2(2, 1)
    job = Job(a.gpus)
    from gameoflife import _native as N
    from gameoflife.engine import GolEngine
    rank, world, local = job.rank, job.world, job.local
    info = N.runtime_info()
    ilv = N_layout(a.board)

    W = H = a.board
    parity = Parity()
    # Every GPU runs the same sequence at every N: the 65536^2 measurement
    # (BASELINE.json configs[2]) first, then the 262144^2 workload.  At N = 1
    # the 65536^2 board comes first because a board allocated after the
    # 16 GiB one was freed stepped ~5 % slower (scripts/alloc_order.py); at
    # N > 1 each rank creates its shard and its RCCL communicator first (the
    # communicator setup idles the GPU for up to a second), then runs the same
    # 65536^2 measurement.  Either way the timed window then starts from its
    # own settle (fresh_window).
    secondary = None
    if world == 1 and not a.no_secondary:
        secondary = secondary_run(GolEngine, a, local, parity)
        secondary["configs1_4096"] = small_board_run(GolEngine, local, parity)
        secondary["configs0_default_board"] = default_board_run(GolEngine, local, parity)
    row0, rows = N.shard_rows(H, rank, world)
    eng = GolEngine(W, H, topology="torus", rule="life", device=local, row0=row0, rows=rows)
    eng.set_tuning(band_rows=a.band, gens_per_pass=a.gpp)
    if world > 1:
        job.join(eng, N)
        if not a.no_secondary:
            secondary = secondary_run(GolEngine, a, local, parity if rank == 0 else None)
            secondary["note"] = f"measured on rank {rank}'s GPU; each of the {world} ranks ran it on its own GPU"

    dt, kms, launches, gcov, clk, hs = fresh_window(eng, job, a.steps, a.warmup, a.hash, 100.0, 12)
    stats = timed_run.stats
    e1 = a.warmup + a.steps
    rank_times = list(getattr(timed_run, "rank_times", []))
    ranks_diag = rank_table(job, N, stats, dt if world == 1 else rank_times[rank], info) if world > 1 else None
    if hs is not None:
        parity.sequence("fused per-generation hashes of the W + K generations (global: shard partials "
                        "summed by gol_comm_allreduce_u64 at N > 1)",
                        (W, H), 1, eng.allreduce_u64(hs) if world > 1 else hs)
    parity.board("gol_hash of the board after the W + K generations (summed over the ranks)", (W, H), e1,
                 global_hash(eng, job))
    eng_info = {g: eng.occupancy(g) for g in range(1, 13)}
    plan = eng.pass_plan(min(a.steps, 1024), hashes=a.hash)
    value = W * H * a.steps / dt / 1e9
    hashed = None
    if not a.hash:
        # the same workload with the fused per-generation state hash (the
        # parity contract's output: one u64 per generation),
        # continuing from the board the timed run left; at N > 1 the shards'
        # per-generation partials are summed over the ring (RCCL all-reduce)
        dth, kmsh, lh, gh, ch, hh = timed_run(eng, job, a.steps, a.warmup, True)
        parity.sequence("fused per-generation hashes of the hashed window (global: shard partials summed "
                        "by gol_comm_allreduce_u64 at N > 1)", (W, H), e1 + 1,
                        eng.allreduce_u64(hh) if world > 1 else hh)
        parity.board("gol_hash of the board after the hashed window", (W, H), 2 * e1, global_hash(eng, job))
        hplan = eng.pass_plan(min(a.steps, 1024), hashes=True)
        vh = W * H * a.steps / dth / 1e9
        hashed = {"value": round(vh, 2), "unit": "GCUPS", "ms_per_step": round(dth / a.steps * 1e3, 4),
                  "frac_of_unhashed": round(vh / value, 4), "pass_plan": hplan,
                  "roofline": roofline(kmsh, lh, gh, W * rows if world == 1 else W * max(rows - round(2 * gh / max(lh, 1)), 0),
                                       hplan, f"{W}x{rows}", "N1" if world == 1 else "ring", True, ch)}
    # dominant kernel: the whole-shard (N=1) or interior-rows (N>1) launch of a
    # pass; G = generations that launch advances (the library's choice when --gpp 0)
    G = gcov / launches if launches else (a.gpp or 1)  # mean depth of the timed passes
    if world == 1:
        roof = roofline(kms, launches, gcov, W * rows, plan, f"{W}x{rows}", "N1", a.hash, clk)
    else:
        roof = roofline(kms, launches, gcov, W * max(rows - round(2 * G), 0), plan, f"{W}x{rows}", "ring", a.hash,
                        clk)
    if roof is not None:
        roof["kernel"] = kernel_label(eng_info, plan, ilv)
    ring = None
    if world == 1 and not a.no_ring and not a.hash:
        ring = ring_schedule_runs(GolEngine, N, a, local, eng, W, H, parity)
    absorbed, absorbed_last = N.absorbed()
    runtime = dict(info, rccl_statuses_absorbed=absorbed)
    if absorbed:
        runtime["rccl_status_last"] = absorbed_last
    if ranks_diag is not None:
        runtime["same_on_all_ranks"] = len({tuple(r[10:13]) for r in ranks_diag}) == 1
    out = {
        "metric": "cell updates/sec (GCUPS) at 1/2/4/8 MI355X + % of HBM roofline",
        "value": round(value, 2),
        "unit": "GCUPS",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(dt / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u32 (bit-packed cells, bitwise ops)",
        "data": "synthetic (splitmix64 Bernoulli(0.5) board, seed 0x5EED)",
        "config": {"workload": f"{W}x{H} torus B3/S23 row-sharded over {world} GPU(s) "
                               f"(BASELINE.json configs[3]; N=1 = whole board on one GPU)",
                   "board": [W, H], "rule": "B3/S23", "topology": "torus",
                   "parallelism": ("single GPU, whole board (no halo exchange)" if world == 1 else
                                   f"row-block x{world}, G-deep RCCL halo send/recv per pass (ring over xGMI)"),
                   "generations_per_pass": round(G, 3), "band_rows": a.band or "auto",
                   "fused_hash": bool(a.hash),
                   "layout": {1: "row-major", 2: "pairs"}.get(ilv, ilv),
                   "window": "seed, 100 ms untimed settle, re-seed, W warm-up + K timed generations"},
        "roofline": roof,
        "parity": parity.report(),
        "runtime": runtime,
    }
    if world > 1:
        rt = rank_times
        d = ranks_diag
        out["ranks"] = {"ms_per_step": [round(x / a.steps * 1e3, 4) for x in rt],
                        "rows": [N.shard_rows(H, r, world)[1] for r in range(world)],
                        "gcups": [round(W * N.shard_rows(H, r, world)[1] * a.steps / x / 1e9, 2)
                                  for r, x in enumerate(rt)],
                        "interior_ms_per_launch": [round(r[1] / 1e6 / max(r[2], 1), 4) for r in d],
                        "exchange_ms_per_pass": [round(r[3] / 1e6 / max(r[4], 1), 4) for r in d],
                        "boundary_ms_per_pass": [round(r[5] / 1e6 / max(r[6], 1), 4) for r in d],
                        "exchange_exposed_ms_per_pass": [round(r[13] / 1e6 / max(r[4], 1), 4) for r in d],
                        "pass_tail_ms_per_pass": [round(r[14] / 1e6 / max(r[6], 1), 4) for r in d],
                        "halo_bytes_per_pass": [round((r[7] + r[8]) / max(r[2], 1)) for r in d],
                        "passes": [r[2] for r in d],
                        "rccl_statuses_absorbed": [r[9] for r in d],
                        "hip_runtime_version": [r[10] for r in d],
                        "rccl_version": [r[11] for r in d],
                        "note": "each rank's own timed window (clock stopped at its own sync; value uses the max); "
                                "interior = the launch overlapping the exchange; exchange = comm-stream HIP events "
                                "around the RCCL group, waiting for a late peer included; exposed / tail = how long "
                                "after the interior launch the exchange / the boundary launch ended (the pass's "
                                "critical path beyond the interior)"}
    if hashed is not None:
        out["with_state_hash"] = hashed
    if ring is not None:
        out["ring_schedule_n1"] = ring
    job.barrier()
    if rank == 0 and secondary is not None:
        out["secondary"] = secondary
    if world > 1 and not a.no_fault:
        # The drill runs after the measured windows, on a ring rebuilt around a
        # lost rank -- a path that has not met every multi-GPU fabric yet.  A
        # watchdog keeps it from costing the line: past --fault-timeout every
        # rank stops, rank 0 printing the line with the drill marked timed out.
        import copy
        import threading

        # What the watchdog prints is fixed before the drill starts: the
        # drill keeps appending to parity.checks on the main thread, which
        # the timer thread must not read mid-update.
        line_before = copy.deepcopy(dict(out, parity=parity.report()))
        failed_before = parity.failed(a.allow_unchecked)

        def give_up():
            msg = f"fault drill did not finish within {a.fault_timeout:.0f} s"
            if rank == 0:
                errs = drill_errors(job)
                fr = {"status": "timed out", "timeout_s": a.fault_timeout,
                      "note": "ranks whose drill raised (rank_errors) left their peers waiting in a collective; "
                              "each also reports on its own stderr"}
                if errs:
                    fr["rank_errors"] = errs
                line = dict(line_before, fault_recovery=fr)
                line["parity_failed"] = failed_before + [msg] + [f"fault drill raised on rank {r}: {e}"
                                                                 for r, e in sorted(errs.items())]
                line["parity_ok"] = False
                os.write(result_fd, (json.dumps(line) + "\n").encode())
            print(f"bench.py rank {rank}: {msg}", file=sys.stderr, flush=True)
            os._exit(4)

        watchdog = threading.Timer(a.fault_timeout, give_up)
        watchdog.daemon = True
        watchdog.start()
        fault, eng = fault_drill(job, N, GolEngine, eng, a, W, H, local, parity)
        watchdog.cancel()
        if fault is not None:
            out["fault_recovery"] = fault
    if eng is not None:
        eng.close()
    if rank == 0 and world == 1 and not a.no_cpu:
        out["cpu_baseline"] = cpu_baseline(W, a.cpu_seconds)
    # The compact parity verdict closes the line, so a tail of it always shows
    # the headline's own check; a failed (or, without --allow-unchecked,
    # unchecked) window fails the run after the line is printed.
    failed = parity.failed(a.allow_unchecked)
    out["parity_failed"] = failed
    out["parity_ok"] = not failed
    if rank == 0:
        sys.stdout.flush()
        os.write(result_fd, (json.dumps(out) + "\n").encode())
    if failed:
        print(f"bench.py rank {rank}: parity failed: {failed}", file=sys.stderr, flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()
