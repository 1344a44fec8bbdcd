"""Instruction census of a kernel's largest loop in a hipcc -S listing.

    python scripts/isa_loop.py build/asm/g7.s multistep_hg_kernelILi2ELi7ELb1ELb0ELb0ELb1

Finds the symbol whose mangled name contains the pattern, takes its longest
backward branch (the unrolled row loop) and prints VALU / SALU / branch
counts and the most frequent opcodes.  Used to check what an addressing or
loop-shape change does to the steady-state instruction mix before spending
GPU time on it (DESIGN.md "Row addressing")."""
import collections
import re
import sys


def census(path, pattern):
    s = open(path).read()
    m = re.search(r"^(_Z\S*%s\S*):" % re.escape(pattern), s, re.M)
    if not m:
        raise SystemExit(f"no symbol matching {pattern}")
    i = m.start()
    body = s[i:s.index(".Lfunc_end", i)].split("\n")
    labels = {l.split(":")[0]: k for k, l in enumerate(body) if re.match(r"\.LBB\d+_\d+:", l)}
    best = None
    for k, l in enumerate(body):
        b = re.search(r"s_c?branch\w*\s+(\.LBB\d+_\d+)", l)
        if b and b.group(1) in labels and labels[b.group(1)] < k:
            n = k - labels[b.group(1)]
            if not best or n > best[0]:
                best = (n, labels[b.group(1)], k)
    _, a, b = best
    cnt = collections.Counter()
    for l in body[a:b + 1]:
        t = l.strip().split()
        if t and not t[0].startswith((".", ";")) and not t[0].endswith(":"):
            cnt[t[0]] += 1
    return m.group(1), cnt


def main():
    name, cnt = census(sys.argv[1], sys.argv[2])
    tot = lambda f: sum(v for k, v in cnt.items() if f(k))
    print(name)
    print("VALU", tot(lambda k: k.startswith("v_")), "SALU", tot(lambda k: k.startswith("s_")),
          "branches", tot(lambda k: "branch" in k), "loads", tot(lambda k: "load" in k),
          "scratch", tot(lambda k: k.startswith("scratch_")))
    for k, v in cnt.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 14):
        print(f"{v:6d} {k}")


if __name__ == "__main__":
    main()
