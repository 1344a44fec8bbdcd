#!/usr/bin/env python3
"""bench.py -- generation-step throughput (GCUPS) + HBM roofline fraction.

Workload (BASELINE.json configs[3], DESIGN.md "Measurement"): a 262144 x
262144 torus, B3/S23, Bernoulli(0.5) splitmix64 board (seed 0x5EED),
row-sharded over N GPUs (strong scaling; N = 1 runs the whole board on one
GPU).  A "step" is one generation of the whole board.  At N = 1 the
single-GPU roofline run of configs[2] (65536^2) is measured too and reported
under "secondary".

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

value = W*H*K / max-over-ranks wall time of the K timed generations (GCUPS),
with the board already resident in HBM.  roofline.achieved = algorithmic bytes
(0.25 B per cell-update: 1 bit read + 1 bit written) per step-kernel launch /
the launch's average duration from HIP events on the launch stream.
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
DEFAULT_GPP = 0  # generations per HBM pass: 0 = libgol's pass planner (gol_pass_plan, DESIGN.md "Pass planner")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: 60 timed generations = 2 x 6 + 6 x 8 passes at 262144^2 (the planner's choice)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=6)
    ap.add_argument("--board", type=int, default=262144, help="board edge (cells)")
    ap.add_argument("--band", type=int, default=0, help="rows per band (0 = auto)")
    ap.add_argument("--gpp", type=int, default=DEFAULT_GPP,
                    help="generations fused per HBM pass (temporal blocking depth 1..8; 0 = automatic)")
    ap.add_argument("--hash", action="store_true", help="fuse the per-generation state hash")
    ap.add_argument("--no-secondary", action="store_true")
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
    eng.step(warmup, hashes=with_hash)
    eng.sync()
    eng.profile(True)
    eng.profile_reset()
    barrier(dist, world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.step(steps, hashes=with_hash)
    eng.sync()
    torch.cuda.synchronize()
    barrier(dist, world)
    dt = time.perf_counter() - t0
    kms, launches, gens = eng.profile_read()
    eng.profile(False)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt, kms, launches, gens


def cpu_baseline(width, seconds):
    """Oracle (bit-packed, bit-sliced, OpenMP) on a bounded sample of the same
    workload: a torus of the same width and 1024 rows, run for ~`seconds`."""
    from oracle import oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    threads = min(threads, os.cpu_count() or threads)
    H = 1024
    board = O.seed_packed(width, H, 0x5EED)
    O.run_packed(board, width, 1, nthreads=threads, want_hashes=False)  # warm
    gens, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        board, _ = O.run_packed(board, width, 4, nthreads=threads, want_hashes=False)
        gens += 4
    dt = time.perf_counter() - t0
    return {"value": round(width * H * gens / dt / 1e9, 3), "unit": "GCUPS", "cores": threads,
            "kind": "port",
            "sample": f"oracle_run_packed (oracle/gol_oracle.c), {width}x{H} torus B3/S23 slice of "
                      f"the same workload, {gens} generations in {dt:.1f} s, {threads} OpenMP threads"}


def roofline(kms, launches, gens_covered, cells_per_gen_per_launch):
    """Algorithmic bytes per launch (0.25 B per cell-update x cells x the
    generations one launch advances) / the launch's average duration."""
    if not launches:
        return None
    avg_s = kms / 1e3 / launches
    gpl = gens_covered / launches
    algo = cells_per_gen_per_launch * gpl * BYTES_PER_CELL_UPDATE
    ach = algo / avg_s / 1e9
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
            "avg_launch_ms": round(avg_s * 1e3, 4), "launches": launches,
            "generations_per_launch": gpl, "algorithmic_bytes_per_launch": algo}


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


def traffic_key(W, H, world, gpp, steps):
    """profiles/pmc_traffic.json key: fixed depth G, or the automatic plan of
    `steps` generations (scripts/prof_run.py runs the same plan)."""
    return f"{W}x{H}/N{world}/G{gpp}" if gpp else f"{W}x{H}/N{world}/auto{steps}"


# Issue-cost model of the multi-generation kernel (DESIGN.md "Roofline"):
# VALU instructions per 32-cell word and generation in the loop of
# multistep_hg_kernel<2, G, LIFE> on the pair layout (from its ISA), and the
# measured cycles per wave64 instruction on one SIMD (profiles/r01_valu_op_costs.txt).
# per 32-cell word and generation in the hg kernel's loop (full-sum rule circuit,
# scripts/isa_loop.py census: 800 VALU per 6-row unroll at G = 6 = 72 DPP + 72
# alignbit + 648 bitop3 + loop overhead), issue costs from op_cost.hip
VALU_MIX = {"v_bitop3_b32": (9, 2.3), "v_alignbit_b32": (1, 4.1), "v_mov_b32_dpp": (1, 4.3)}
SIMDS = 256 * 4
CLOCK_GHZ = 2.4  # MI355X_MICROARCH.md max clock


def valu_roofline(gcups):
    """Cell-update rate the VALU issue model allows at the max clock (every
    SIMD issuing the loop's instruction mix back to back), and the fraction
    of it the run reached.  Halo lanes and band halo rows are overheads
    counted against the kernel, not removed from the peak."""
    cycles = sum(n * c for n, c in VALU_MIX.values())
    peak = SIMDS * CLOCK_GHZ * 1e9 / cycles * 64 * 32 / 1e9
    return {"bound": "valu", "instructions_per_word_generation": {k: n for k, (n, _) in VALU_MIX.items()},
            "cycles_per_word_generation": round(cycles, 2), "clock_ghz": CLOCK_GHZ,
            "peak_gcups": round(peak, 1), "frac": round(gcups / peak, 4),
            "source": "profiles/r01_valu_op_costs.txt (scripts/micro/op_cost.hip)"}


def pmc_traffic(workload_key):
    """HBM bytes per launch measured with rocprofv3 --pmc (profiles/pmc_traffic.json,
    written by scripts/pmc_traffic.py with the gfx950 FETCH_SIZE x2 correction)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(workload_key)
    except (OSError, ValueError):
        return None


def secondary_run(GolEngine, torch, dist, a, local):
    """BASELINE.json configs[2]: the 65536^2 single-GPU roofline run."""
    S = 65536
    with GolEngine(S, S, topology="torus", rule="life", device=local) as e2:
        e2.set_tuning(band_rows=a.band, gens_per_pass=a.gpp)
        e2.seed(0x5EED)
        # >= 10 warm-up and >= 100 timed
        # generations, rounded up to whole 6-generation passes
        n2, w2 = max(a.steps, 102), max(a.warmup, 12)
        dt2, kms2, l2, g2 = timed_run(e2, torch, dist, 1, n2, w2, a.hash)
        # the same board one generation per HBM pass: the pure bandwidth case
        # (north_star: >= 70 % of peak HBM bandwidth at 65536^2)
        e2.set_tuning(band_rows=a.band, gens_per_pass=1)
        e2.seed(0x5EED)
        dt1, kms1, l1, g1 = timed_run(e2, torch, dist, 1, n2, w2, a.hash)
    r2 = with_traffic(roofline(kms2, l2, g2, S * S), traffic_key(S, S, 1, a.gpp, n2))
    r1 = with_traffic(roofline(kms1, l1, g1, S * S), f"{S}x{S}/N1/G1")
    return {"workload": "65536x65536 torus B3/S23 on 1 GPU (BASELINE.json configs[2])",
            "value": round(S * S * n2 / dt2 / 1e9, 2), "unit": "GCUPS", "steps": n2, "warmup": w2,
            "ms_per_step": round(dt2 / n2 * 1e3, 4), "roofline": r2,
            "single_generation_passes": {"value": round(S * S * n2 / dt1 / 1e9, 2), "unit": "GCUPS",
                                         "ms_per_step": round(dt1 / n2 * 1e3, 4), "roofline": r1}}


def with_traffic(r, key):
    """Add the PMC-measured HBM bytes per launch (and the bandwidth they
    imply at the measured launch time) to a roofline object."""
    if r is None:
        return None
    t = pmc_traffic(key)
    if t is not None:
        r["traffic"] = t.get("hbm_bytes_per_launch")
        r["traffic_source"] = t.get("source")
        if r["traffic"]:
            gbs = r["traffic"] / (r["avg_launch_ms"] * 1e-3) / 1e9
            r["measured_hbm_gbs"] = round(gbs, 1)
            r["measured_hbm_frac"] = round(gbs / HBM_PEAK_GBS, 4)
    return r


def main():
    a = parse()
    torch, dist, rank, world, local = dist_setup(a.gpus)
    from gameoflife import _native as N
    from gameoflife.engine import GolEngine

    W = H = a.board
    # configs[2] (65536^2, N = 1 only) first: a board allocated after the
    # 16 GiB one was freed stepped ~5 % slower (scripts/alloc_order.py).
    secondary = None
    if rank == 0 and world == 1 and not a.no_secondary:
        secondary = secondary_run(GolEngine, torch, dist, a, local)
    row0, rows = N.shard_rows(H, rank, world)
    eng = GolEngine(W, H, topology="torus", rule="life", device=local, row0=row0, rows=rows)
    eng.set_tuning(band_rows=a.band, gens_per_pass=a.gpp)
    if world > 1:
        uid = N.unique_id() if rank == 0 else bytes(N.GOL_UNIQUE_ID_BYTES)
        t = torch.tensor(list(uid), dtype=torch.uint8)
        dist.broadcast(t, 0)
        eng.comm_init(bytes(t.tolist()), rank, world)
    eng.seed(0x5EED)

    dt, kms, launches, gcov = timed_run(eng, torch, dist, world, a.steps, a.warmup, a.hash)
    eng_info = {g: eng.occupancy(g) for g in range(1, 9)}
    plan = eng.pass_plan(min(a.steps, 1024), hashes=a.hash)
    value = W * H * a.steps / dt / 1e9
    hashed = None
    if world == 1 and not a.hash:
        # the same workload with the fused per-generation state hash (the
        # parity contract's output: one u64 per generation),
        # continuing from the board the timed run left
        dth, _, _, _ = timed_run(eng, torch, dist, world, a.steps, 1, True)
        hashed = {"value": round(W * H * a.steps / dth / 1e9, 2), "unit": "GCUPS",
                  "ms_per_step": round(dth / a.steps * 1e3, 4),
                  "pass_plan": eng.pass_plan(min(a.steps, 1024), hashes=True)}
    # dominant kernel: the whole-shard (N=1) or interior-rows (N>1) launch of a
    # pass; G = generations that launch advances (the library's choice when --gpp 0)
    G = gcov / launches if launches else (a.gpp or 1)  # mean depth of the timed passes
    cells = W * (rows if world == 1 else max(rows - round(2 * G), 0))
    roof = roofline(kms, launches, gcov, cells)
    key = traffic_key(W, H, world, a.gpp, a.steps)
    if roof is not None:
        roof["kernel"] = kernel_label(eng_info, plan)
        roof["pass_plan"] = plan
        if "multistep_hg_kernel<2," in roof["kernel"] and N.pair_layout(W):
            # per-launch rate of the dominant kernel, not the wall-clock value
            roof["valu"] = valu_roofline(cells * gcov / launches / (roof["avg_launch_ms"] * 1e-3) / 1e9)
        with_traffic(roof, key)
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
                   "parallelism": f"row-block x{world}, RCCL halo send/recv",
                   "generations_per_pass": round(G, 3), "band_rows": a.band or "auto",
                   "fused_hash": bool(a.hash)},
        "roofline": roof,
    }
    if hashed is not None:
        out["with_state_hash"] = hashed
    eng.close()

    if rank == 0 and world == 1:
        if secondary is not None:
            out["secondary"] = secondary
        if not a.no_cpu:
            out["cpu_baseline"] = cpu_baseline(W, a.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
