"""Per-kernel register and occupancy table from `make asm`'s
-Rpass-analysis=kernel-resource-usage remarks.

    python scripts/resource_usage.py akka-game-of-life_amd/build/asm/resource-usage-g*.txt [filter]

Kernel names are shortened to kernel<VEC,G,LIFE,HASH,CLIPPED,PAIRS>."""
import re
import sys

KEYS = ("VGPRs", "TotalSGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]")


def short(name):
    m = re.search(r"\d+([a-z_]+_kernel)I(.*)EEvNS_10StepParamsE", name)
    if not m:
        return name
    args = re.findall(r"Li(\d+)E|Lb([01])E", m.group(2))
    return f"{m.group(1)}<{','.join(a or b for a, b in args)}>"


def main():
    paths = [a for a in sys.argv[1:] if a.endswith(".txt")]
    filt = [a for a in sys.argv[1:] if not a.endswith(".txt")]
    rows, cur = [], None
    for p in paths:
        for line in open(p):
            m = re.search(r"Function Name: (\S+)", line)
            if m:
                cur = {"name": short(m.group(1))}
                rows.append(cur)
                continue
            for k in KEYS:
                m = re.search(r"remark:\s+%s: (\d+)" % re.escape(k), line)
                if m and cur is not None:
                    cur[k] = int(m.group(1))
    print(f"{'kernel<VEC,G,LIFE,HASH,CLIPPED,PAIRS>':48s} VGPR SGPR scratch waves/SIMD")
    for r in rows:
        if filt and not any(f in r["name"] for f in filt):
            continue
        print(f"{r['name']:48s} {r.get('VGPRs', 0):4d} {r.get('TotalSGPRs', 0):4d} {r.get(KEYS[2], 0):7d} "
              f"{r.get(KEYS[3], 0):4d}")


if __name__ == "__main__":
    main()
