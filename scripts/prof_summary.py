#!/usr/bin/env python3
"""Summarise a scripts/gpu_prof.sh run (gpurun_out/prof) into profiles/:

* <tag>_kernel_stats.csv      rocprofv3 --stats of the bench command (verbatim)
* <tag>_kernel_trace.txt      per-(kernel, grid) dispatch durations of the same
                              command, beside the bench's own HIP-event numbers
* <tag>_bench.json            the bench line printed under rocprofv3 and unprofiled

Per-launch PMC numbers (HBM bytes, clock, VALU issue) come from
scripts/gpu_pmc.sh + scripts/pmc_launch.py (profiles/pmc_launch.json).

    python3 scripts/prof_summary.py [prof_dir] [tag]
"""
import csv
import json
import os
import shutil
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STEP_KERNELS = ("step_kernel", "multistep_kernel", "multistep_hg_kernel")


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def pmc_per_dispatch(path, counter):
    out = []
    for r in rows(path):
        if r["Counter_Name"] == counter and any(k in r["Kernel_Name"] for k in STEP_KERNELS):
            out.append(float(r["Counter_Value"]))
    return out


def main():
    prof = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "prof")
    tag = sys.argv[2] if len(sys.argv) > 2 else "r01"
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)

    shutil.copy(os.path.join(prof, "bench_trace", "bench_kernel_stats.csv"),
                os.path.join(dst, f"{tag}_kernel_stats.csv"))
    benches = {}
    for name in ("bench_under_rocprof.json", "bench.json"):
        with open(os.path.join(prof, name)) as f:
            lines = [ln for ln in f if ln.startswith("{")]
        benches[name] = json.loads(lines[-1])
    with open(os.path.join(dst, f"{tag}_bench.json"), "w") as f:
        json.dump(benches, f, indent=1)

    trace = rows(os.path.join(prof, "bench_trace", "bench_kernel_trace.csv"))
    trace.sort(key=lambda r: int(r["Start_Timestamp"]))
    groups = defaultdict(list)  # (kernel, grid) -> durations in dispatch order
    for r in trace:
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        groups[(r["Kernel_Name"], int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]))].append(dur)
    b = benches["bench_under_rocprof.json"]
    lines = [f"rocprofv3 --kernel-trace --stats -- python3 bench.py --steps {b['steps']} --warmup {b['warmup']}",
             "per (kernel, grid): dispatches, mean / median / min ms", ""]
    for (name, gx, gy), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"{name:40s} grid=({gx},{gy}) n={len(d):3d} mean={statistics.mean(d):.4f} "
                     f"median={statistics.median(d):.4f} min={min(d):.4f}")
    lines += ["", "bench.py HIP-event numbers from the same run (timed region only) beside the trace:"]

    def instance(G, hashed):
        # multistep_hg_kernel<2, G, LIFE, HASH, torus, ILV = 2, not whole-row>
        # (step_kernel<4, ...> at G = 1); round 5's names lack the last argument
        h = "true" if hashed else "false"
        if G == 1:
            return f"step_kernel<4, true, {h}, false, 2>"
        return f"multistep_hg_kernel<2, {G}, true, {h}, false, 2"


    # Dispatches in time order.  Round 4's window (bench.py fresh_window):
    # seed, untimed settle passes, seed again, the warm-up pass, the timed
    # passes; the hashed window follows with no seed.  The timed launches are
    # found by walking the trace from the main board's second seed.
    order = [(r["Kernel_Name"], int(r["Grid_Size_X"]),
              (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6) for r in trace]
    big_seed = max((gx for n, gx, _ in order if "seed_kernel" in n), default=0)
    seeds = [i for i, (n, gx, _) in enumerate(order) if "seed_kernel" in n and gx == big_seed]

    def whole_board(G, hashed):
        cands = [gx for (name, gx, gy) in groups if instance(G, hashed) in name]
        return max(cands) if cands else None

    def walk(start, plan, hashed, warmup):
        """Durations of the timed launches after dispatch `start` (the warm-up
        pass first, when there is one), and the index after them."""
        i, out = start, []
        steps = ([warmup] if warmup and warmup <= 12 else []) + list(plan)
        for k, G in enumerate(steps):
            gx = whole_board(G, hashed)
            if gx is None:
                return None, start
            while i < len(order) and not (instance(G, hashed) in order[i][0] and order[i][1] == gx):
                i += 1
            if i == len(order):
                return None, start
            if k >= len(steps) - len(plan):
                out.append(order[i][2])
            i += 1
        return out, i

    main_t, after = walk(seeds[1], b.get("pass_plan") or b["roofline"].get("pass_plan"), False,
                         b.get("warmup")) if len(seeds) > 1 else (None, 0)
    hrec = b.get("with_state_hash")
    hash_t = walk(after, hrec["pass_plan"], True, b.get("warmup"))[0] if hrec and main_t else None
    for label, rec, t in (("main workload", b, main_t), ("with_state_hash", hrec, hash_t)):
        if not rec or not rec.get("roofline"):
            continue
        ro = rec["roofline"]
        lines.append(f"  {label:16s} bench avg_launch_ms={ro.get('avg_launch_ms')} launches={ro.get('launches')}"
                     + (f"   rocprof, the same timed launches: mean={statistics.mean(t):.4f} ms "
                        f"({', '.join(f'{x:.4f}' for x in t)})" if t else ""))
    lines.append("(the timed launches are picked from the trace in dispatch order: from the main board's second")
    lines.append(" seed (the re-seed after the untimed settle), the warm-up pass, then the timed passes; the")
    lines.append(" hashed window's follow them; the instances' other launches at the same grids are the settle")
    lines.append(" passes and the N = 1 ring-schedule runs)")
    with open(os.path.join(dst, f"{tag}_kernel_trace.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))

    pdir = os.path.join(dst, f"{tag}_pmc")
    os.makedirs(pdir, exist_ok=True)
    for d in sorted(os.listdir(prof)):
        src = os.path.join(prof, d, "run_counter_collection.csv")
        if d.startswith("pmc_") and os.path.exists(src):
            shutil.copy(src, os.path.join(pdir, f"{d}.csv"))


if __name__ == "__main__":
    main()
