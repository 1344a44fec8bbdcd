#!/usr/bin/env python3
"""Reconcile the two clock readings of the bench's timed launches (VERDICT
r02 item 4): one `rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU` pass over the
driver's exact command (`bench.py --steps 20 --warmup 5`), whose output line
carries the in-kernel probe clock of the same launches (held_clock.ghz).

For the headline window's timed launches -- the last len(plan) step-kernel
dispatches before the run's first gol_hash (bench.py's parity check right
after the window) -- it writes the PMC clock (GRBM_GUI_ACTIVE / 8 XCDs /
launch time), the time-weighted mean over the plan, the probe clock from the
same run's JSON line, and the VALU per word-generation; likewise for the
hashed window (before the second gol_hash).

    python3 scripts/clock_reconcile.py gpurun_out/clk profiles/r03_clock_reconcile.txt
"""
import csv
import json
import os
import sys
from collections import defaultdict


def dispatches(path):
    d = defaultdict(lambda: {"name": "", "grid": 0, "t": 0.0, "c": defaultdict(float)})
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            e = d[int(r["Dispatch_Id"])]
            e["name"] = r["Kernel_Name"]
            e["grid"] = int(r["Grid_Size"])
            e["t"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            e["c"][r["Counter_Name"]] += float(r["Counter_Value"])
    return [d[k] for k in sorted(d)]


def pick(ds, n, k):
    """The timed launches of window k: the last n step-kernel dispatches
    before the k-th gol_hash (hash_kernel) of the headline board -- bench.py
    hashes the board right after each window for its parity check.  Round 4
    checks the 65536^2 windows too, so only the hashes of the 16x larger
    262144^2 board count (the hash grid is capped, so it is told apart by its
    duration).  (rocprofv3 -T truncates the kernel names to their base
    names, so the order is the key.)"""
    hs = [i for i, e in enumerate(ds) if e["name"].startswith("hash_kernel")]
    longest = max(ds[i]["t"] for i in hs)
    hashes = [i for i in hs if ds[i]["t"] >= 0.5 * longest]
    end = hashes[k]
    steps = [i for i in range(end) if e_is_step(ds[i])]
    return [ds[i] for i in steps[-n:]]


def e_is_step(e):
    return e["name"].startswith(("multistep_hg_kernel", "multistep_kernel", "step_kernel"))


def main():
    src, dst = sys.argv[1], sys.argv[2]
    ds = dispatches(os.path.join(src, "bench_clock", "bench_counter_collection.csv"))
    with open(os.path.join(src, "bench_under_pmc.json")) as f:
        b = json.loads([ln for ln in f if ln.startswith("{")][-1])
    W, H = b["config"]["board"]
    lines = [f"rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU -- python3 bench.py --steps {b['steps']} "
             f"--warmup {b['warmup']}  (one run: counters and the bench line of the same launches)", ""]
    for k, (label, rec) in enumerate((("headline window", b), ("hashed window", b.get("with_state_hash")))):
        ro = rec["roofline"]
        plan = ro["pass_plan"]
        got = pick(ds, len(plan), k)
        if len(got) != len(plan):
            lines.append(f"{label}: timed launches not found in the trace")
            continue
        lines.append(f"{label}: plan {plan}")
        tw = 0.0
        for G, e in zip(plan, got):
            clk = e["c"]["GRBM_GUI_ACTIVE"] / 8 / e["t"] / 1e9
            valu = e["c"]["SQ_INSTS_VALU"] * 64 / (W * H / 32 * G)
            tw += clk * e["t"]
            lines.append(f"  G={G:2d} launch {e['t'] * 1e3:7.3f} ms  PMC clock {clk:.3f} GHz  "
                         f"VALU/word-gen {valu:.3f}")
        t = sum(e["t"] for e in got)
        hc = ro.get("held_clock", {})
        lines.append(f"  time-weighted PMC clock {tw / t:.3f} GHz; in-kernel probe of the same launches "
                     f"(bench line held_clock.ghz) {hc.get('ghz')} GHz; bench avg_launch_ms {ro['avg_launch_ms']} "
                     f"vs PMC-run mean {t / len(got) * 1e3:.4f} ms")
        lines.append("")
    lines.append("PMC clock = GRBM_GUI_ACTIVE / 8 XCDs / launch time (MI355X_MICROARCH.md 'DVFS give-back'); "
                 "the probe = sampled workgroups' s_memtime / s_memrealtime ticks (gol_profile_clock)")
    with open(dst, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
