"""CPU: the B3/S23 gate circuit of the step kernels
(`rule_b3s23_fullsum`, akka-game-of-life_amd/csrc/gol_stencil.h, used by
`rule_hg` and `rule_words` on tori), and the row-pair-shared circuit of
`multistep_hg_kernel` (`pair_sum` + `rule_b3s23_pair`), are the rule.

The kernel's truth-table constants are read from the header and evaluated
as `v_bitop3_b32` does (bit a<<2 | b<<1 | c of the table), first on every
one of the 2^7 inputs (three rows' 2-bit horizontal sums + the centre cell),
then word-parallel over a packed torus against the oracle's step
(rule: NextStateCellGathererActor.scala:42-44 read as B3/S23)."""
import os
import re

import numpy as np
import pytest

from oracle import oracle as O

HDR = os.path.join(os.path.dirname(os.path.dirname(__file__)), "akka-game-of-life_amd", "csrc", "gol_stencil.h")


def _consts():
    src = open(HDR).read()
    out = {}
    for name in ("kXor3", "kMaj", "kXnor3", "kNotAllEq", "kRuleT1", "kRuleT2", "kRuleOut",
                 "kPairT1", "kPairT2", "kPairT3", "kPairOut"):
        m = re.search(r"constexpr uint32_t %s = (0x[0-9A-Fa-f]+);" % name, src)
        assert m, name
        out[name] = int(m.group(1), 16)
    return out


K = _consts()


def bitop3(a, b, c, t):
    """v_bitop3_b32 on scalars or uint32 arrays."""
    a, b, c = (np.asarray(x, dtype=np.uint32) for x in (a, b, c))
    r = np.zeros(np.broadcast(a, b, c).shape, dtype=np.uint32)
    full = np.uint32(0xFFFFFFFF)
    for i in range(8):
        if (t >> i) & 1:
            r |= (a if i & 4 else a ^ full) & (b if i & 2 else b ^ full) & (c if i & 1 else c ^ full)
    return r


def rule_hg(a0, a1, c0, c1, b0, b1, r):
    """rule_b3s23_fullsum, gate for gate."""
    e1 = bitop3(a0, c0, b0, K["kXnor3"])
    e2 = bitop3(a0, c0, b0, K["kNotAllEq"])
    f1 = bitop3(a1, c1, b1, K["kXnor3"])
    f2 = bitop3(a1, c1, b1, K["kNotAllEq"])
    t1 = bitop3(e1, e2, f2, K["kRuleT1"])
    t2 = bitop3(e1, r, t1, K["kRuleT2"])
    return bitop3(e2, f1, t2, K["kRuleOut"])


def test_circuit_exhaustive():
    """Every combination of three 2-bit row sums (h = W + C + E in 0..3)
    and the centre bit: next = S == 3 or (S == 4 and alive), S = 9-cell sum."""
    for ha in range(4):
        for hc in range(4):
            for hb in range(4):
                for alive in range(2):
                    if alive and hc == 0:
                        continue  # the centre is one of the three cells summed into hc
                    S = ha + hc + hb
                    want = 1 if S == 3 or (S == 4 and alive) else 0
                    got = int(rule_hg(ha & 1, ha >> 1, hc & 1, hc >> 1, hb & 1, hb >> 1, alive)) & 1
                    assert got == want, (ha, hc, hb, alive)


@pytest.mark.parametrize("W,H,seed", [(64, 40, 1), (256, 33, 2), (96, 17, 3)])
def test_circuit_word_parallel_matches_oracle(W, H, seed):
    """Row-major words, horizontal sums from funnel shifts (torus wrap), the
    gate circuit per word: equals the oracle's packed step."""
    packed = O.seed_packed(W, H, seed)
    nw = packed.shape[1]
    x = packed.astype(np.uint64)
    # west neighbour bit of cell i is cell i-1: shift left by one with the
    # previous word's top bit carried in; east mirrors it.
    prev = np.roll(x, 1, axis=1)
    nxt = np.roll(x, -1, axis=1)
    west = ((x << 1) | (prev >> 31)) & 0xFFFFFFFF
    east = ((x >> 1) | (nxt << 31)) & 0xFFFFFFFF
    c = x & 0xFFFFFFFF
    h0 = bitop3(west, c, east, K["kXor3"])
    h1 = bitop3(west, c, east, K["kMaj"])
    up0, up1 = np.roll(h0, 1, axis=0), np.roll(h1, 1, axis=0)
    dn0, dn1 = np.roll(h0, -1, axis=0), np.roll(h1, -1, axis=0)
    got = rule_hg(up0, up1, h0, h1, dn0, dn1, c)
    want = O.step_packed(packed, W, O.TORUS, O.LIFE)
    assert nw == W // 32
    assert (got == want[:, :nw]).all()


@pytest.mark.parametrize("W,H,seed", [(64, 40, 4), (160, 21, 5)])
def test_circuit_vertical_first_matches_oracle(W, H, seed):
    """The vertical-first order (column 3-sums, then the columns left and
    right of each cell: rule_words) feeds the same circuit."""
    packed = O.seed_packed(W, H, seed)
    nw = packed.shape[1]
    c = packed.astype(np.uint32)
    a, b = np.roll(c, 1, axis=0), np.roll(c, -1, axis=0)
    v0 = bitop3(a, c, b, K["kXor3"]).astype(np.uint64)
    v1 = bitop3(a, c, b, K["kMaj"]).astype(np.uint64)

    def west(v):
        return ((v << 1) | (np.roll(v, 1, axis=1) >> 31)) & 0xFFFFFFFF

    def east(v):
        return ((v >> 1) | (np.roll(v, -1, axis=1) << 31)) & 0xFFFFFFFF

    got = rule_hg(west(v0), west(v1), v0, v1, east(v0), east(v1), c)
    assert (got == O.step_packed(packed, W, O.TORUS, O.LIFE)[:, :nw]).all()


def pair_sum(a0, a1, b0, b1):
    """pair_sum: the binary sum P = a + b of two rows' 2-bit sums."""
    a0, a1, b0, b1 = (np.asarray(x, dtype=np.uint32) for x in (a0, a1, b0, b1))
    k = a0 & b0
    return a0 ^ b0, bitop3(a1, b1, k, K["kXor3"]), bitop3(a1, b1, k, K["kMaj"])


def rule_pair(p0, p1, p2, x0, x1, alive):
    """rule_b3s23_pair, gate for gate."""
    g1 = bitop3(p0, x0, alive, K["kPairT1"])
    g2 = bitop3(p1, p2, g1, K["kPairT2"])
    g3 = bitop3(p2, x1, g2, K["kPairT3"])
    return bitop3(g3, alive, g1, K["kPairOut"])


def test_pair_circuit_exhaustive():
    """Both rows of a pair: row m adds h(m-1) to P = h(m) + h(m+1) (its centre
    in the first term of P), row m+1 adds h(m+2) to P = h(m) + h(m+1) (its
    centre in the second).  Every 2-bit row sum and centre bit."""
    for hx in range(4):
        for hc in range(4):
            for ho in range(4):
                for alive in range(2):
                    if alive and hc == 0:
                        continue
                    S = hx + hc + ho
                    want = 1 if S == 3 or (S == 4 and alive) else 0
                    for first, second in ((hc, ho), (ho, hc)):
                        p = pair_sum(first & 1, first >> 1, second & 1, second >> 1)
                        got = int(rule_pair(*p, hx & 1, hx >> 1, alive)) & 1
                        assert got == want, (hx, hc, ho, alive, first, second)


@pytest.mark.parametrize("W,H,seed", [(64, 40, 6), (96, 18, 7)])
def test_pair_circuit_word_parallel_matches_oracle(W, H, seed):
    """Even rows form P with the row below, odd rows reuse the P of the row
    above (the kernel's schedule, H even): equals the oracle's packed step."""
    packed = O.seed_packed(W, H, seed)
    nw = packed.shape[1]
    x = packed.astype(np.uint64)
    west = ((x << 1) | (np.roll(x, 1, axis=1) >> 31)) & 0xFFFFFFFF
    east = ((x >> 1) | (np.roll(x, -1, axis=1) << 31)) & 0xFFFFFFFF
    c = x & 0xFFFFFFFF
    h0 = bitop3(west, c, east, K["kXor3"])
    h1 = bitop3(west, c, east, K["kMaj"])
    got = np.zeros_like(h0)
    for m in range(0, H, 2):
        n1, u, d = (m + 1) % H, (m - 1) % H, (m + 2) % H
        P = pair_sum(h0[m], h1[m], h0[n1], h1[n1])
        got[m] = rule_pair(*P, h0[u], h1[u], c[m])
        got[n1] = rule_pair(*P, h0[d], h1[d], c[n1])
    want = O.step_packed(packed, W, O.TORUS, O.LIFE)
    assert (got == want[:, :nw]).all()
