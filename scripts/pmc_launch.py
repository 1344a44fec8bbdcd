#!/usr/bin/env python3
"""Summarise scripts/gpu_pmc.sh (gpurun_out/pmc) into profiles/pmc_launch.json:
per step-kernel launch of each (shape, mode, pass depth G, hash) --

  hbm_bytes        = (2 x FETCH_SIZE + WRITE_SIZE) x 1024   (MI355X_MICROARCH.md
                     "HBM": FETCH_SIZE and WRITE_SIZE are KiB; on gfx950
                     FETCH_SIZE reads half the bytes of a wide streaming read)
  clock_ghz        = GRBM_GUI_ACTIVE / 8 XCDs / launch time  ("DVFS")
  valu_per_word_gen = SQ_INSTS_VALU x 64 lanes / (32-bit words x G)
  launch_ms        = mean duration of those launches in the clock pass

Launches: the step-kernel dispatches with the largest grid (the whole shard,
or a ring shard's interior rows), the warm-up pass's dropped.  The CSVs are
copied to profiles/<tag>_pmc/; keys already in profiles/pmc_launch.json and
not measured in this run are kept.

    python3 scripts/pmc_launch.py [gpurun_out/pmc] [tag]
"""
import csv
import json
import os
import shutil
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STEP = ("step_kernel", "multistep_kernel", "multistep_hg_kernel")


def dispatches(path):
    """{dispatch id: (grid, duration s, {counter: value})} of the step kernels."""
    d = defaultdict(lambda: [0, 0.0, defaultdict(float)])
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            if not any(k in r["Kernel_Name"] for k in STEP):
                continue
            e = d[int(r["Dispatch_Id"])]
            e[0] = int(r["Grid_Size"])
            e[1] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            e[2][r["Counter_Name"]] += float(r["Counter_Value"])
    return d


def main_launches(path):
    d = dispatches(path)
    if not d:
        return []
    big = max(e[0] for e in d.values())
    out = [d[k] for k in sorted(d) if d[k][0] == big]
    return out[1:]  # drop the warm-up pass


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pmc")
    tag = sys.argv[2] if len(sys.argv) > 2 else "r02"
    path = os.path.join(ROOT, "profiles", "pmc_launch.json")
    out = {}
    if os.path.exists(path):  # earlier runs' keys stay; keys measured again are replaced
        with open(path) as f:
            out = json.load(f)
    keys = sorted({d.split("__")[0] for d in os.listdir(src) if "__" in d and os.path.isdir(os.path.join(src, d))})
    for key in keys:
        shape, mode, g, h = key.split("_")
        W, H = (int(v) for v in shape.split("x"))
        G, hashed = int(g[1:]), int(h[1:])
        csvs = {p: os.path.join(src, f"{key}__{p}", "run_counter_collection.csv") for p in ("fetch", "write", "clock")}
        if not all(os.path.exists(c) for c in csvs.values()):
            continue
        fe, wr, ck = (main_launches(csvs[p]) for p in ("fetch", "write", "clock"))
        n = min(len(fe), len(wr), len(ck))
        if n == 0:
            continue
        fetch = 2 * statistics.fmean(e[2]["FETCH_SIZE"] for e in fe[:n]) * 1024
        write = statistics.fmean(e[2]["WRITE_SIZE"] for e in wr[:n]) * 1024
        t = statistics.fmean(e[1] for e in ck[:n])
        clk = statistics.fmean(e[2]["GRBM_GUI_ACTIVE"] / 8 / e[1] / 1e9 for e in ck[:n])
        rows = H - 2 * G if mode == "ring" else H
        words = rows * (W // 32)
        valu = statistics.fmean(e[2]["SQ_INSTS_VALU"] for e in ck[:n]) * 64 / (words * G)
        plane = W * rows / 8
        out[f"{shape}/{mode}/G{G}/h{hashed}"] = {
            "launch_ms": round(t * 1e3, 4),
            "hbm_bytes": round(fetch + write),
            "fetch_bytes": round(fetch),
            "write_bytes": round(write),
            "planes_read": round(fetch / plane, 3),
            "planes_written": round(write / plane, 3),
            "clock_ghz": round(clk, 3),
            "valu_per_word_gen": round(valu, 3),
            "cells_per_launch": W * rows,
            "generations_per_launch": G,
            "launches": n,
            "source": f"profiles/{tag}_pmc/{key}__*.csv (scripts/gpu_pmc.sh: separate rocprofv3 --pmc passes "
                      f"over scripts/prof_run.py {shape} {G}{' --hash' if hashed else ''}"
                      f"{' --ring' if mode == 'ring' else ''})"}
        dst = os.path.join(ROOT, "profiles", f"{tag}_pmc")
        os.makedirs(dst, exist_ok=True)
        for p, c in csvs.items():
            shutil.copy(c, os.path.join(dst, f"{key}__{p}.csv"))
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    for k, v in sorted(out.items()):
        print(f"{k:32s} {v['launch_ms']:8.4f} ms  hbm={v['hbm_bytes'] / 1e9:7.3f} GB "
              f"(read {v['planes_read']:.3f} + write {v['planes_written']:.3f} planes)  "
              f"clock={v['clock_ghz']:.3f} GHz  VALU/word-gen={v['valu_per_word_gen']:.2f}")


if __name__ == "__main__":
    main()
