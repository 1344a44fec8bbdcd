#!/usr/bin/env python3
"""Summarise a scripts/gpu_prof.sh run (gpurun_out/prof) into profiles/:

* <tag>_kernel_stats.csv      rocprofv3 --stats of the bench command (verbatim)
* <tag>_kernel_trace.txt      per-(kernel, grid) dispatch durations of the same
                              command, beside the bench's own HIP-event numbers
* <tag>_bench.json            the bench line printed under rocprofv3 and unprofiled
* pmc_traffic.json            HBM bytes per step launch from separate --pmc passes

HBM bytes (MI355X_MICROARCH.md "HBM"): FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reads exactly half the bytes of a 16-B-per-lane
streaming read, so hbm = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.  The G=1
kernel's WRITE_SIZE equals one plane exactly, which checks the unit.

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
GENS = {262144: 60, 65536: 102}  # timed generations of bench.py's two boards


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
    groups = defaultdict(list)
    for r in trace:
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        groups[(r["Kernel_Name"], int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]))].append(dur)
    b = benches["bench_under_rocprof.json"]
    lines = ["rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 60 --warmup 6",
             "per (kernel, grid): dispatches, mean / median / min ms", ""]
    for (name, gx, gy), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"{name:40s} grid=({gx},{gy}) n={len(d):3d} mean={statistics.mean(d):.4f} "
                     f"median={statistics.median(d):.4f} min={min(d):.4f}")
    lines += ["", "bench.py HIP-event numbers from the same run (timed region only):",
              f"  main workload   avg_launch_ms={b['roofline']['avg_launch_ms']} launches={b['roofline']['launches']}",
              f"  secondary       avg_launch_ms={b['secondary']['roofline']['avg_launch_ms']} "
              f"launches={b['secondary']['roofline']['launches']}",
              "(rocprof's counts include the warm-up launch of each workload)"]
    with open(os.path.join(dst, f"{tag}_kernel_trace.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))

    traffic = {}
    for edge in (262144, 65536):
        for g in (0, 1):
            fdir = os.path.join(prof, f"pmc_FETCH_SIZE_{edge}_g{g}", "run_counter_collection.csv")
            wdir = os.path.join(prof, f"pmc_WRITE_SIZE_{edge}_g{g}", "run_counter_collection.csv")
            if not (os.path.exists(fdir) and os.path.exists(wdir)):
                continue
            fetch = pmc_per_dispatch(fdir, "FETCH_SIZE")
            write = pmc_per_dispatch(wdir, "WRITE_SIZE")
            # g = 0: the automatic pass plan of the bench's generation count
            # (mixed depths: per-launch means), g = 1: single-generation passes
            gens = GENS[edge] if g == 0 else 60
            n = min(len(fetch), len(write))
            fetch, write = fetch[:n], write[:n]
            G = gens / n if g == 0 else 1  # generations per launch
            f_b, w_b = 2 * statistics.fmean(fetch) * 1024, statistics.fmean(write) * 1024
            hbm = f_b + w_b
            plane = edge * edge / 8
            key = f"{edge}x{edge}/N1/auto{gens}" if g == 0 else f"{edge}x{edge}/N1/G1"
            traffic[key] = {
                "hbm_bytes_per_launch": round(hbm),
                "fetch_bytes_per_launch": round(f_b),
                "write_bytes_per_launch": round(w_b),
                "planes_read": round(f_b / plane, 3),
                "planes_written": round(w_b / plane, 3),
                "generations_per_launch": round(G, 3),
                "algorithmic_bytes_per_launch": edge * edge * 0.25 * G,
                "hbm_bytes_per_cell_generation": round(hbm / (edge * edge * G), 4),
                "launches_measured": n,
                "source": f"profiles/{tag}_pmc (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, "
                          f"scripts/prof_run.py {edge} {gens} {g}; FETCH_SIZE x2 gfx950 correction)"}
    with open(os.path.join(dst, "pmc_traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1)
    pdir = os.path.join(dst, f"{tag}_pmc")
    os.makedirs(pdir, exist_ok=True)
    for d in sorted(os.listdir(prof)):
        src = os.path.join(prof, d, "run_counter_collection.csv")
        if d.startswith("pmc_") and os.path.exists(src):
            shutil.copy(src, os.path.join(pdir, f"{d}.csv"))
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
