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
with the board already resident in HBM.

roofline: the dominant kernel (the whole-shard launch at
N = 1, a shard's interior-rows launch at N > 1) is bound by VALU issue, not by
HBM -- temporal blocking fuses 6-8 generations per pass over the plane.  So:
  * roofline.bound = "valu": achieved = cell-updates per second of that launch
    (cells x generations per launch / its mean HIP-event duration), peak = the
    VALU-issue ceiling of the kernel's loop mix at the guide's 2.4 GHz max
    clock, frac = achieved / peak; roofline.held_clock prices the same launches
    at the clock they actually held (in-kernel probe, gol_profile_clock) as an
    issue-efficiency diagnostic, with the PMC clock (profiles/) beside it;
  * roofline.traffic = PMC HBM bytes per launch, and roofline.hbm the physical
    HBM bandwidth that implies against the 8 TB/s spec;
  * roofline.hbm_effective = SURVEY.md section 8(d)'s 2 bits per cell-update,
    counted per generation: above 1 by construction of temporal blocking.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
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
# LIFE> on the pair layout (scripts/isa_loop.py census: at G = 6, 800 VALU per
# 6-row unroll = 648 bitop3 + 72 alignbit + 72 DPP + loop overhead) and the
# measured cycles per wave64 instruction on one SIMD (profiles/r01_valu_op_costs.txt).
VALU_MIX = {"v_bitop3_b32": (9, 2.3), "v_alignbit_b32": (1, 4.1), "v_mov_b32_dpp": (1, 4.3)}
# The fused hash adds one v_mad_u64_u32 per word and generation (DESIGN.md "State hash").
VALU_MIX_HASH = dict(VALU_MIX, v_mad_u64_u32=(1, 4.6))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: 60 timed generations = 2 x 6 + 6 x 8 passes at 262144^2 (the planner's choice)
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
    return ap.parse_args()


def dist_setup(n):
    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n:
        raise SystemExit(f"--gpus {n} but WORLD_SIZE={world}")
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(local)
    return torch, dist, rank, world, local


def barrier(dist, world):
    if world > 1:
        dist.barrier()


def timed_run(eng, torch, dist, world, steps, warmup, with_hash):
    """W untimed + K timed generations.  Returns (seconds, kernel ms,
    launches, generations covered by them, probe clock GHz, hashes): hashes
    = the W + K per-generation partial hashes of this shard when with_hash."""
    hw = eng.step(warmup, hashes=with_hash) if warmup > 0 else None
    eng.sync()
    eng.profile(True)
    eng.profile_reset()
    barrier(dist, world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ht = eng.step(steps, hashes=with_hash)
    eng.sync()
    torch.cuda.synchronize()
    # the clock stops when this rank's work is done; the closing barrier and
    # the max over ranks then give the job's time (a gloo barrier costs
    # ~1 ms, a real share of an N = 8 rank's 20-step window)
    dt = time.perf_counter() - t0
    barrier(dist, world)
    kms, launches, gens = eng.profile_read()
    clock = eng.profile_clock()  # GHz the timed launches ran at (in-kernel probe)
    eng.profile(False)
    if world > 1:
        # every rank's own time (rank order) -> the job's time is their max
        t = torch.zeros(world, dtype=torch.float64)
        t[dist.get_rank()] = dt
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        timed_run.rank_times = [float(x) for x in t.tolist()]
        dt = max(timed_run.rank_times)
    hashes = None
    if with_hash:
        import numpy as np
        hashes = np.concatenate([h for h in (hw, ht) if h is not None]).astype(np.uint64)
    return dt, kms, launches, gens, clock, hashes


GOLDEN_SEED = 0x5EED


def golden_path(W):
    return os.path.join("tests", "golden", f"bench_{W}.json")


def golden_hashes(W, H):
    """Global state hashes of the bench board (W x H torus, B3/S23, seed
    0x5EED) at epochs 0, 1, ..., from tests/golden/bench_<W>.json -- written by
    tests/golden/make_bench_golden.py with the CPU oracle (a data file: bench
    never runs the oracle to check itself).  None if there is no table."""
    try:
        with open(os.path.join(ROOT, golden_path(W))) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("board") != [W, H] or d.get("seed") != GOLDEN_SEED or d.get("rule") != "B3/S23":
        return None
    return [int(x, 16) for x in d["hashes"]]


def global_hash(eng, world):
    """The whole board's state hash: gol_hash of every shard, summed over the
    ranks with gol_comm_allreduce_u64 (RCCL) -- the hash is a sum mod 2^64, so
    the N shards' partials add up to the N = 1 value."""
    import numpy as np
    h = np.array([eng.hash()], dtype=np.uint64)
    if world > 1:
        h = eng.allreduce_u64(h)
    return int(h[0])


class Parity:
    """bench.py's self-check against the committed golden hashes: every rank's
    shard is checked at every N, so the multi-GPU line records whether the RCCL
    halo exchange kept the board bit-exact (CellActor.scala:71-77,
    NextStateCellGathererActor.scala:32-36 are the exchange it replaces)."""

    def __init__(self, W, H):
        self.golden = golden_hashes(W, H)
        self.source = golden_path(W)
        self.checks = []

    def _golden(self, epoch):
        return self.golden[epoch] if self.golden is not None and epoch < len(self.golden) else None

    def board(self, what, epoch, value):
        g = self._golden(epoch)
        self.checks.append({"what": what, "epoch": epoch, "hash": f"{value:#018x}",
                            "golden": None if g is None else f"{g:#018x}",
                            "match": None if g is None else value == g})

    def sequence(self, what, first_epoch, values):
        gs = [self._golden(first_epoch + k) for k in range(len(values))]
        known = [(first_epoch + k, int(v), g) for k, (v, g) in enumerate(zip(values, gs)) if g is not None]
        bad = [e for e, v, g in known if v != g]
        self.checks.append({"what": what, "epochs": [first_epoch, first_epoch + len(values) - 1],
                            "checked": len(known), "mismatched_epochs": bad[:16],
                            "last_hash": f"{int(values[-1]):#018x}" if len(values) else None,
                            "match": (not bad) if known else None})

    def report(self):
        ms = [c["match"] for c in self.checks]
        return {"golden": f"{self.source} (CPU oracle, tests/golden/make_bench_golden.py; "
                          "parity unpinned: the reference ships no vectors)" if self.golden else None,
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


def cpu_baseline(width, seconds):
    """Oracle (bit-packed, bit-sliced, OpenMP) on a bounded sample of the same
    workload: a torus of the same width and 1024 rows, run for ~`seconds`.
    The reported value uses the CPU share the harness grants the job
    (OMP_NUM_THREADS: 16 threads per GPU on the pool's boxes); a shorter
    sample on every core of sched_getaffinity (all
    host cores) is reported beside it when that is more threads."""
    from oracle import oracle as O
    affinity = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(share, affinity) if share > 0 else affinity
    H = 1024
    v, gens, dt = _cpu_rate(O, width, H, threads, seconds)
    out = {"value": round(v, 3), "unit": "GCUPS", "cores": threads,
           "kind": "port", "nproc": os.cpu_count(), "affinity": affinity, "cpu_model": cpu_model(),
           "threads_source": "OMP_NUM_THREADS (the job's CPU share)" if share > 0 else "sched_getaffinity",
           "sample": f"oracle_run_packed (oracle/gol_oracle.c, bit-sliced, OpenMP), {width}x{H} torus B3/S23 "
                     f"slice of the same workload, {gens} generations in {dt:.1f} s on {threads} threads"}
    quota = cgroup_cpus()
    if quota:
        out["cgroup_cpu_quota"] = quota
    if affinity > threads:
        va, ga, dta = _cpu_rate(O, width, H, affinity, max(seconds / 3, 1.0))
        out["all_affinity"] = {"value": round(va, 3), "unit": "GCUPS", "cores": affinity,
                               "sample": f"same slice, {ga} generations in {dta:.1f} s on {affinity} threads",
                               "note": (f"the job's cgroup grants {quota:g} CPUs: {affinity} threads time-slice on "
                                        "them" if quota and quota < affinity else "every core of sched_getaffinity")}
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
        if pmc:
            r["traffic"] = round(pmc["hbm_bytes"])
            r["measured_hbm_gbs"] = round(pmc["hbm_bytes"] / avg_s / 1e9, 1)
            r["measured_hbm_frac"] = round(pmc["hbm_bytes"] / avg_s / 1e9 / HBM_PEAK_GBS, 4)
            r["traffic_source"] = "profiles/pmc_launch.json " + ", ".join(pmc["keys"])
        return r
    mix = VALU_MIX_HASH if hashed else VALU_MIX
    # frac: against the VALU-issue ceiling at the guide's max clock (2.4 GHz,
    # MI355X_MICROARCH.md) -- the peak the chip is specified for.  The clock
    # these launches actually held (in-kernel probe, gol_profile_clock) only
    # prices the separate issue-efficiency diagnostic under held_clock.
    peak_max, cycles = valu_peak_gcups(mix, CLOCK_MAX_GHZ)
    r = {"bound": "valu", "achieved": round(gcups, 1), "peak": round(peak_max, 1), "unit": "GCUPS",
         "frac": round(gcups / peak_max, 4), "traffic": round(pmc["hbm_bytes"]) if pmc else None,
         "peak_clock_ghz": CLOCK_MAX_GHZ,
         "valu": {"instructions_per_word_generation": {k: n for k, (n, _) in mix.items()},
                  "cycles_per_word_generation": round(cycles, 2),
                  "measured_valu_per_word_generation": round(pmc["valu_per_word_gen"], 2) if pmc else None,
                  "source": "loop census scripts/isa_loop.py; issue costs profiles/r01_valu_op_costs.txt"},
         **common}
    held = {"clock_pmc_ghz": round(pmc["clock_ghz"], 3) if pmc else None}
    if clock:
        peak_held, _ = valu_peak_gcups(mix, clock)
        held.update({"ghz": round(clock, 3), "peak_at_held_clock": round(peak_held, 1),
                     "issue_efficiency": round(gcups / peak_held, 4),
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


def kernel_label(info, depths):
    """Name of the kernel instances the timed passes launch (depths: the pass
    plan, gol_pass_plan): the strip width (gol_occupancy) gives the words per
    lane; multi-generation passes at 8-byte lanes or narrower run the
    horizontal-first kernel (gol_capi.cpp kernel_variant)."""
    gs = sorted(set(depths)) or [1]
    waves, strip = info.get(gs[-1], (0, 0))
    if gs == [1]:
        vec = strip // 64 if strip else "VEC"
        return f"gol::dev::step_kernel<{vec},LIFE>"
    vec = strip // 62 if strip else 0
    name = "multistep_hg_kernel" if vec in (1, 2) and os.environ.get("GOL_STENCIL_VARIANT", "2") != "1" \
        else "multistep_kernel"
    return f"gol::dev::{name}<{vec or 'VEC'},{'|'.join(map(str, gs))},LIFE> ({waves} waves/CU resident)"


def settle(eng, ms, with_hash, chunk):
    """Step `eng` untimed until `ms` of GPU time has passed: after an idle
    gap (context creation, seeding) the chip's clock dips and recovers over
    ~15-20 ms of work (profiles/r02_warmup_curve.txt), longer than a short
    window at 0.04 ms per generation."""
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        eng.step(chunk, hashes=with_hash)
        eng.sync()


def secondary_run(GolEngine, torch, dist, a, local):
    """BASELINE.json configs[2]: the 65536^2 single-GPU roofline run.

    Two windows on the same board: SURVEY.md section 8(d)'s minimum (>= 10
    warm-up, >= 100 timed generations: 4 ms at 65536^2, inside the clock's
    recovery after the idle gap) as "short_window", and the reported value
    over >= 1024 generations after 50 ms of untimed steps, when the clock has
    settled (profiles/r02_warmup_curve.txt)."""
    S = 65536
    out = {"workload": "65536x65536 torus B3/S23 on 1 GPU (BASELINE.json configs[2])"}
    with GolEngine(S, S, topology="torus", rule="life", device=local) as e2:
        e2.set_tuning(band_rows=a.band, gens_per_pass=a.gpp)
        e2.seed(0x5EED)
        n_s, w_s = max(a.steps, 102), max(a.warmup, 12)
        dt_s, _, _, _, _, _ = timed_run(e2, torch, dist, 1, n_s, w_s, a.hash)
        settle(e2, 50.0, a.hash, 64)
        n2 = max(a.steps, 1024)
        dt2, kms2, l2, g2, c2, _ = timed_run(e2, torch, dist, 1, n2, 0, a.hash)
        plan2 = e2.pass_plan(n2, hashes=a.hash)
        # the same board one generation per HBM pass: the pure bandwidth case
        # (north_star: >= 70 % of peak HBM bandwidth at 65536^2)
        e2.set_tuning(band_rows=a.band, gens_per_pass=1)
        e2.seed(0x5EED)
        settle(e2, 50.0, a.hash, 16)
        n1 = max(a.steps, 256)
        dt1, kms1, l1, g1, c1, _ = timed_run(e2, torch, dist, 1, n1, 0, a.hash)
    shape = f"{S}x{S}"
    r2 = roofline(kms2, l2, g2, S * S, plan2, shape, "N1", a.hash, c2)
    r1 = roofline(kms1, l1, g1, S * S, [1] * n1, shape, "N1", a.hash, c1)
    out.update({
        "value": round(S * S * n2 / dt2 / 1e9, 2), "unit": "GCUPS", "steps": n2, "warmup": "50 ms settled",
        "ms_per_step": round(dt2 / n2 * 1e3, 4), "roofline": r2,
        "short_window": {"value": round(S * S * n_s / dt_s / 1e9, 2), "unit": "GCUPS", "steps": n_s,
                         "warmup": w_s, "ms_per_step": round(dt_s / n_s * 1e3, 4),
                         "note": "fresh seed right after context creation: inside the clock's recovery"},
        "single_generation_passes": {"value": round(S * S * n1 / dt1 / 1e9, 2), "unit": "GCUPS", "steps": n1,
                                     "warmup": "50 ms settled", "ms_per_step": round(dt1 / n1 * 1e3, 4),
                                     "roofline": r1,
                                     # the same bytes over the wall-clock time per generation
                                     # (launch gaps included), beside the kernel-time frac
                                     "hbm_frac_from_ms_per_step": round(
                                         S * S * BYTES_PER_CELL_UPDATE / (dt1 / n1) / 1e9 / HBM_PEAK_GBS, 4)}})
    return out


def ring_schedule_runs(GolEngine, N, torch, dist, a, local, eng, W, H):
    """N = 1 only: the row-sharded (RCCL ring) schedule on this GPU, as a 1-rank
    self-ring (gol_capi.cpp one_pass: interior launch || G-row halo
    ncclSend/ncclRecv to itself, then the boundary rows on the edge stream).
    (1) the whole board, (2) one rank's shard of the N = 8 decomposition
    (262144 x 32768): what each of 8 ranks computes, without the xGMI latency
    of a real ring.  Both after 50 ms of untimed steps: after the GPU idles
    (here: the shard's allocation) the first ~15-20 ms of launches run 10-25 %
    slower while the power management settles (profiles/r02_warmup_curve.txt),
    which a few generations of a 0.08 ms-per-generation shard do not cover."""
    out = {}
    warm = "50 ms settled"
    eng.comm_init(N.unique_id(), 0, 1)
    eng.seed(0x5EED)
    settle(eng, 50.0, False, 12)
    dt, kms, launches, gcov, _, _ = timed_run(eng, torch, dist, 1, a.steps, a.warmup, False)
    out["whole_board_self_ring"] = {"value": round(W * H * a.steps / dt / 1e9, 2), "unit": "GCUPS",
                                    "warmup": warm, "ms_per_step": round(dt / a.steps * 1e3, 4),
                                    "pass_plan": eng.pass_plan(min(a.steps, 1024))}
    rows8 = H // 8
    with GolEngine(W, H, topology="torus", rule="life", device=local, row0=0, rows=rows8) as e8:
        e8.comm_init(N.unique_id(), 0, 1)  # a 1-rank ring over a shard-sized torus
        # First as an N = 8 rank meets the driver's window (main(), N > 1):
        # the GPU idle while the ranks initialise RCCL, the 65536^2 run, then
        # seed, W warm-up steps and the timed steps, no settle -- like the
        # N = 1 line's own window, so the two compare directly.
        time.sleep(1.0)
        if not a.no_secondary:
            secondary_run(GolEngine, torch, dist, a, local)
        e8.seed(0x5EED)
        dtf, _, _, _, _, _ = timed_run(e8, torch, dist, 1, a.steps, a.warmup, False)
        out["per_rank_shard_driver_window"] = {
            "shard": f"{W}x{rows8} (one rank of N = 8)", "value": round(W * rows8 * a.steps / dtf / 1e9, 2),
            "unit": "GCUPS", "warmup": a.warmup, "ms_per_step": round(dtf / a.steps * 1e3, 4),
            "note": "an N = 8 rank's sequence on this GPU (1 s idle for the communicator setup, the 65536^2 run, "
                    "seed, W warm-up and K timed steps); x 8 / the N = 1 value is the per-cell efficiency that "
                    "run can reach before any xGMI cost"}
        e8.seed(0x5EED)
        settle(e8, 50.0, False, 12)
        dt8, kms8, l8, g8, c8, _ = timed_run(e8, torch, dist, 1, a.steps, a.warmup, False)
        plan8 = e8.pass_plan(min(a.steps, 1024))
    out["per_rank_shard_self_ring"] = {
        "shard": f"{W}x{rows8} (one rank of N = 8)", "value": round(W * rows8 * a.steps / dt8 / 1e9, 2),
        "unit": "GCUPS", "warmup": warm, "ms_per_step": round(dt8 / a.steps * 1e3, 4), "pass_plan": plan8,
        "interior_launch": roofline(kms8, l8, g8, W * max(rows8 - round(2 * g8 / max(l8, 1)), 0), plan8,
                                    f"{W}x{rows8}", "ring", False, c8)}
    return out


def main():
    a = parse()
    # one JSON line on stdout: native libraries (RCCL's version banner at
    # communicator creation) write to fd 1, so it points at stderr until the
    # result is printed on the saved descriptor
    sys.stdout.flush()
    result_fd = os.dup(1)
    os.dup2(2, 1)
    torch, dist, rank, world, local = dist_setup(a.gpus)
    from gameoflife import _native as N
    from gameoflife.engine import GolEngine

    W = H = a.board
    # Every GPU runs the same sequence at every N: the 65536^2 measurement
    # (BASELINE.json configs[2]) first, then the 262144^2 workload.  At N = 1
    # the 65536^2 board comes first because a board allocated after the
    # 16 GiB one was freed stepped ~5 % slower (scripts/alloc_order.py); at
    # N > 1 each rank creates its shard and its RCCL communicator first (the
    # communicator setup idles the GPU for up to a second), then runs the same
    # 65536^2 measurement, so the sharded window starts from a GPU as busy as
    # the N = 1 window does (after an idle gap the first ~15-20 ms of launches
    # run 10-25 % slower, profiles/r02_warmup_curve.txt).
    secondary = None
    if world == 1 and not a.no_secondary:
        secondary = secondary_run(GolEngine, torch, dist, a, local)
    row0, rows = N.shard_rows(H, rank, world)
    eng = GolEngine(W, H, topology="torus", rule="life", device=local, row0=row0, rows=rows)
    eng.set_tuning(band_rows=a.band, gens_per_pass=a.gpp)
    if world > 1:
        uid = N.unique_id() if rank == 0 else bytes(N.GOL_UNIQUE_ID_BYTES)
        t = torch.tensor(list(uid), dtype=torch.uint8)
        dist.broadcast(t, 0)
        eng.comm_init(bytes(t.tolist()), rank, world)
        if not a.no_secondary:
            secondary = secondary_run(GolEngine, torch, dist, a, local)
            secondary["note"] = f"measured on rank {rank}'s GPU; each of the {world} ranks ran it on its own GPU"
    eng.seed(GOLDEN_SEED)
    parity = Parity(W, H)

    dt, kms, launches, gcov, clk, hs = timed_run(eng, torch, dist, world, a.steps, a.warmup, a.hash)
    e1 = a.warmup + a.steps
    rank_times = list(getattr(timed_run, "rank_times", []))
    if hs is not None:
        parity.sequence("fused per-generation hashes of the W + K generations (global: shard partials "
                        "summed by gol_comm_allreduce_u64 at N > 1)",
                        1, eng.allreduce_u64(hs) if world > 1 else hs)
    parity.board("gol_hash of the board after the W + K generations (summed over the ranks)", e1,
                 global_hash(eng, world))
    eng_info = {g: eng.occupancy(g) for g in range(1, 13)}
    plan = eng.pass_plan(min(a.steps, 1024), hashes=a.hash)
    value = W * H * a.steps / dt / 1e9
    hashed = None
    if not a.hash:
        # the same workload with the fused per-generation state hash (the
        # parity contract's output: one u64 per generation),
        # continuing from the board the timed run left; at N > 1 the shards'
        # per-generation partials are summed over the ring (RCCL all-reduce)
        dth, kmsh, lh, gh, ch, hh = timed_run(eng, torch, dist, world, a.steps, a.warmup, True)
        parity.sequence("fused per-generation hashes of the hashed window (global: shard partials summed "
                        "by gol_comm_allreduce_u64 at N > 1)", e1 + 1, eng.allreduce_u64(hh) if world > 1 else hh)
        parity.board("gol_hash of the board after the hashed window", 2 * e1, global_hash(eng, world))
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
        roof["kernel"] = kernel_label(eng_info, plan)
    ring = None
    if world == 1 and not a.no_ring and not a.hash:
        ring = ring_schedule_runs(GolEngine, N, torch, dist, a, local, eng, W, H)
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
                   "fused_hash": bool(a.hash)},
        "roofline": roof,
        "parity": parity.report(),
    }
    if world > 1:
        rt = rank_times
        out["ranks"] = {"ms_per_step": [round(x / a.steps * 1e3, 4) for x in rt],
                        "rows": [N.shard_rows(H, r, world)[1] for r in range(world)],
                        "gcups": [round(W * N.shard_rows(H, r, world)[1] * a.steps / x / 1e9, 2)
                                  for r, x in enumerate(rt)],
                        "note": "each rank's own timed window (clock stopped at its own sync); value uses the max"}
    if hashed is not None:
        out["with_state_hash"] = hashed
    if ring is not None:
        out["ring_schedule_n1"] = ring
    eng.close()

    if rank == 0 and secondary is not None:
        out["secondary"] = secondary
    if rank == 0 and world == 1 and not a.no_cpu:
        out["cpu_baseline"] = cpu_baseline(W, a.cpu_seconds)
    if rank == 0:
        sys.stdout.flush()
        os.write(result_fd, (json.dumps(out) + "\n").encode())
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
