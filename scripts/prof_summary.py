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
        # multistep_hg_kernel<2, G, LIFE, HASH, torus, pairs> (step_kernel<2, ...> at G = 1)
        h = "true" if hashed else "false"
        if G == 1:
            return f"step_kernel<2, true, {h}, false, true>"
        return f"multistep_hg_kernel<2, {G}, true, {h}, false, true>"

    def traced(plan, hashed, warmup):
        # The timed launches of a run: in dispatch order, each depth's first
        # launches at the largest grid of its instance (the whole-board
        # launch), after the warm-up's single pass of `warmup` generations
        # (gol_step plans <= 12 generations as one pass).  Returns (mean of
        # the timed launches, mean over every launch of those instances).
        seen = defaultdict(int)
        if warmup and warmup <= 12:
            seen[warmup] = 1
        timed, every = [], []
        for G in plan:
            cands = [(gx, d) for (name, gx, gy), d in groups.items() if instance(G, hashed) in name]
            if not cands:
                return None, None
            gx, d = max(cands, key=lambda c: c[0])
            if seen[G] >= len(d):
                return None, None
            timed.append(d[seen[G]])
            seen[G] += 1
            every.append(statistics.mean(d))
        return statistics.mean(timed), statistics.mean(every)

    for label, rec, hashed in (("main workload", b, False), ("with_state_hash", b.get("with_state_hash"), True)):
        if not rec or not rec.get("roofline"):
            continue
        ro = rec["roofline"]
        plan = rec.get("pass_plan") or ro.get("pass_plan") or b.get("pass_plan")
        t, t_all = traced(plan, hashed, b.get("warmup")) if plan else (None, None)
        lines.append(f"  {label:16s} bench avg_launch_ms={ro.get('avg_launch_ms')} launches={ro.get('launches')}"
                     + (f"   rocprof, the same timed launches: mean={t:.4f} ms"
                        f" (every launch of those instances and grids: {t_all:.4f} ms)" if t else ""))
    lines.append("(the timed launches are picked from the trace in dispatch order: each pass depth's first")
    lines.append(" whole-board launches after the warm-up pass; the instances' later launches at the same grid")
    lines.append(" belong to the N = 1 ring-schedule runs on a settled, sparser board)")
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
