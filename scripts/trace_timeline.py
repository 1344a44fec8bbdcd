#!/usr/bin/env python3
"""Print a rocprofv3 kernel trace as a timeline (start offset, duration, gap
to the previous dispatch's end, kernel, grid) -- for reading the overlap of a
sharded pass (interior launch, RCCL p2p kernel, boundary launch).

    python3 scripts/trace_timeline.py gpurun_out/rank/rank_kernel_trace.csv [first] [count]
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    count = int(sys.argv[3]) if len(sys.argv) > 3 else len(rows)
    t0 = int(rows[first]["Start_Timestamp"]) if rows else 0
    prev_end = None
    for r in rows[first:first + count]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        print(f"{(s - t0) / 1e3:10.1f} us  dur {(e - s) / 1e3:9.1f} us  gap {gap:8.1f} us  "
              f"{r['Kernel_Name'][:60]:60s} grid {r['Grid_Size_X']}")
        prev_end = e if prev_end is None else max(prev_end, e)


if __name__ == "__main__":
    main()
