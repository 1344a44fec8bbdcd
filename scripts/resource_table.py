#!/usr/bin/env python3
"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output: one line per
kernel instance (VGPRs, SGPRs, scratch, waves/SIMD), demangled template args.

    python scripts/resource_table.py build/asm/resource-usage-g10.txt [filter]"""
import re
import sys

FIELDS = ("TotalSGPRs", "VGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]")


def parse(text):
    out, cur = [], None
    for line in text.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            out.append(cur)
            continue
        for f in FIELDS:
            m = re.search(re.escape(f) + r": (\d+)", line)
            if m and cur is not None:
                cur[f] = int(m.group(1))
    return out


def short(name):
    m = re.search(r"dev(\d+)(\w+?)I(.*)EEvNS", name)
    if not m:
        return name
    args = re.findall(r"L([ib])(\d+)E", m.group(3))
    return f"{m.group(2)}<{','.join(v for _, v in args)}>"


if __name__ == "__main__":
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    for k in parse(open(sys.argv[1]).read()):
        s = short(k["name"])
        if flt in s:
            print(f"{s:48s} vgpr {k.get('VGPRs', '?'):>4} sgpr {k.get('TotalSGPRs', '?'):>4} "
                  f"scratch {k.get('ScratchSize [bytes/lane]', '?'):>4} waves {k.get('Occupancy [waves/SIMD]', '?')}")
