"""profiles/copy_peak.json from a scripts/micro/copy_bw run on an MI355X box.

    python scripts/copy_peak.py gpurun_out/r6/copy_bw.txt profiles/r06_copy_bw.txt

Takes the JSON line copy_bw prints last (the best read + write rate over its
variants), adds where it was measured, and writes profiles/copy_peak.json,
which bench.py reports as roofline.copy_peak ("Also report
the measured stream-copy peak")."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src, label = sys.argv[1], sys.argv[2]
    lines = [ln for ln in open(src) if ln.strip()]
    d = json.loads(lines[-1])
    d["measured"] = f"scripts/micro/copy_bw.hip, {label}: best of 20 launches per variant, read + write bytes"
    with open(os.path.join(ROOT, "profiles", "copy_peak.json"), "w") as f:
        json.dump(d, f, indent=1)
        f.write("\n")
    print(json.dumps(d))


if __name__ == "__main__":
    main()
