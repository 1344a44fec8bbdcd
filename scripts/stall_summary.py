#!/usr/bin/env python3
"""Summarise scripts/archive/gpu_stall_pmc.sh (gpurun_out/stall): per config, the
fractions of wave-cycles parked on s_waitcnt (SQ_WAIT_ANY), stalled at issue
(SQ_WAIT_INST_ANY) and issuing (SQ_ACTIVE_INST_ANY / _VALU), over the
largest-grid step-kernel launches (warm-up pass dropped).

    python3 scripts/stall_summary.py [gpurun_out/stall]
"""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/stall"
    for d in sorted(glob.glob(os.path.join(root, "*/"))):
        f = glob.glob(os.path.join(d, "**", "run_counter_collection.csv"), recursive=True)
        if not f:
            continue
        disp = collections.defaultdict(lambda: collections.defaultdict(float))
        grid = {}
        for r in csv.DictReader(open(f[0])):
            if not any(k in r["Kernel_Name"] for k in ("step_kernel", "multistep_hg_kernel")):
                continue
            k = int(r["Dispatch_Id"])
            disp[k][r["Counter_Name"]] += float(r["Counter_Value"])
            grid[k] = int(r["Grid_Size"])
        if not grid:
            continue
        big = max(grid.values())
        tot = collections.defaultdict(float)
        for k in [k for k in sorted(disp) if grid[k] == big][1:]:
            for c, v in disp[k].items():
                tot[c] += v
        wc = tot["SQ_WAVE_CYCLES"] or 1.0
        print(f"{os.path.basename(d.rstrip('/')):28s} wait_any {tot['SQ_WAIT_ANY'] / wc:.3f}  "
              f"wait_inst {tot['SQ_WAIT_INST_ANY'] / wc:.3f}  active {tot['SQ_ACTIVE_INST_ANY'] / wc:.3f}  "
              f"active_valu {tot['SQ_ACTIVE_INST_VALU'] / wc:.3f}  "
              f"valu/salu {tot['SQ_INSTS_VALU'] / max(tot['SQ_INSTS_SALU'], 1):.2f}")


if __name__ == "__main__":
    main()
