#!/usr/bin/env python3
"""Effective clock and VALU issue of the step kernel from one rocprofv3 PMC
pass (scripts/gpu_prof.sh: GRBM_GUI_ACTIVE, SQ_WAVES, SQ_INSTS_VALU,
SQ_ACTIVE_INST_VALU, SQ_WAVE_CYCLES, SQ_BUSY_CYCLES over
scripts/prof_run.py EDGE 60 6: fixed 6-generation passes), per dispatch:

  clock            = GRBM_GUI_ACTIVE / 8 XCDs / kernel time   (MI355X_MICROARCH.md "DVFS")
  VALU/word-gen    = SQ_INSTS_VALU x 64 lanes / (32-bit words x generations)
  issue rate       = SQ_INSTS_VALU / (1024 SIMDs x clock x time)  wave-instr per SIMD-cycle

    python3 scripts/pmc_clock.py counter_collection.csv EDGE [G]
"""
import csv
import sys
from collections import defaultdict


def main():
    path, edge = sys.argv[1], int(sys.argv[2])
    G = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    agg, dur = defaultdict(lambda: defaultdict(float)), {}
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            if "multistep_hg_kernel" not in r["Kernel_Name"]:
                continue
            k = int(r["Dispatch_Id"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[k] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    wordgens = edge // 32 * edge * G
    print(f"# {path}: {edge}^2 torus B3/S23, {G} generations per launch")
    print("dispatch  ms      clock_GHz  VALU_instr/word-gen  wave-instr/SIMD/cycle  GCUPS")
    for k in sorted(agg):
        v, t = agg[k], dur[k]
        clk = v["GRBM_GUI_ACTIVE"] / 8 / t / 1e9
        print(f"{k:8d}  {t * 1e3:6.3f}  {clk:9.3f}  {v['SQ_INSTS_VALU'] * 64 / wordgens:19.2f}  "
              f"{v['SQ_INSTS_VALU'] / (1024 * clk * 1e9 * t):21.3f}  {edge * edge * G / t / 1e9:7.0f}")


if __name__ == "__main__":
    main()
