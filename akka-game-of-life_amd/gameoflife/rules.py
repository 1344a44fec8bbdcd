"""Life-like rules as (birth, survive) 9-bit masks.

Bit k of `birth` set: a dead cell with k live neighbours is born; bit k of
`survive` set: a live cell with k live neighbours stays alive.  The three
named rules come from the reference's rule line and BASELINE.json:

* ``life``          B3/S23 -- the north_star rule (the perf path).
* ``ref-literal``   NextStateCellGathererActor.scala:44 read with a multiset
                    count: a live cell with exactly 3 live neighbours dies,
                    nothing is born (B/S01245678).
* ``ref-effective`` what :42-44 actually computes: the neighbour replies are
                    collapsed by Scala's ``Set.map`` so aliveNeighbours is 0 or
                    1, line 44 never fires, and the board is unchanged
                    (B/S012345678, the identity).
"""
from __future__ import annotations

import re
from dataclasses import dataclass


@dataclass(frozen=True)
class Rule:
    birth: int
    survive: int
    name: str = ""

    def notation(self) -> str:
        b = "".join(str(k) for k in range(9) if (self.birth >> k) & 1)
        s = "".join(str(k) for k in range(9) if (self.survive >> k) & 1)
        return f"B{b}/S{s}"


LIFE = Rule(0x008, 0x00C, "life")
REF_LITERAL = Rule(0x000, 0x1F7, "ref-literal")
REF_EFFECTIVE = Rule(0x000, 0x1FF, "ref-effective")

NAMED = {r.name: r for r in (LIFE, REF_LITERAL, REF_EFFECTIVE)}


def rule_by_name(name: str) -> Rule:
    """'life' | 'ref-literal' | 'ref-effective' | 'B3/S23'-style notation."""
    if name in NAMED:
        return NAMED[name]
    m = re.fullmatch(r"[Bb]([0-8]*)/[Ss]([0-8]*)", name.strip())
    if not m:
        raise ValueError(f"unknown rule {name!r}")
    birth = sum(1 << int(d) for d in m.group(1))
    survive = sum(1 << int(d) for d in m.group(2))
    return Rule(birth, survive, name)
