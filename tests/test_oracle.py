"""CPU tests of the oracle: restatements agree, known-answer patterns hold,
and the committed golden vectors reproduce.  (No GPU.)"""
import ctypes
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


def cells_from(rows):
    return np.array([[int(ch) for ch in r] for r in rows], dtype=np.uint8)


@pytest.mark.parametrize("W,H,topo", [(32, 5, O.TORUS), (64, 64, O.TORUS), (96, 3, O.TORUS),
                                      (32, 1, O.TORUS), (32, 2, O.TORUS), (7, 7, O.REF_CLIPPED),
                                      (33, 40, O.REF_CLIPPED), (100, 65, O.REF_CLIPPED),
                                      (2, 2, O.REF_CLIPPED), (1, 1, O.REF_CLIPPED)])
def test_scalar_packed_numpy_agree(W, H, topo):
    rng = np.random.default_rng(W * 1000 + H)
    rules = [O.LIFE, O.REF_LITERAL, O.REF_EFFECTIVE] + [
        (int(rng.integers(0, 512)), int(rng.integers(0, 512))) for _ in range(4)]
    for rule in rules:
        c = (rng.random((H, W)) < 0.4).astype(np.uint8)
        a = O.step_cells(c, topo, rule)
        b = O.np_step(c, topo, rule)
        p = O.unpack(O.step_packed(O.pack(c), W, topo, rule), W)
        assert (a == b).all() and (a == p).all(), (W, H, topo, rule)


def test_ref_effective_is_identity_and_equals_masks():
    """NextStateCellGathererActor.scala:42-44: Set[Boolean] collapse =>
    aliveNeighbours in {0,1} => line 44 never fires => board unchanged."""
    rng = np.random.default_rng(3)
    for topo, (W, H) in [(O.REF_CLIPPED, (7, 7)), (O.TORUS, (64, 9)), (O.REF_CLIPPED, (30, 11))]:
        c = (rng.random((H, W)) < 0.6).astype(np.uint8)
        lit = O.step_cells(c, topo, mode=O.MODE_REF_EFFECTIVE)
        assert (lit == c).all()
        assert (O.step_cells(c, topo, O.REF_EFFECTIVE) == c).all()
        assert (O.np_step(c, topo, mode=O.MODE_REF_EFFECTIVE) == c).all()


def test_ref_literal_hand_worked():
    """Line 44 with a multiset count: a live cell with exactly 3 live
    neighbours dies, nothing else changes.  Reference geometry 3x3 board
    (4x4 cells), neighbours only from [0,3)x[0,3)."""
    c = cells_from(["1100",
                    "1100",
                    "0001",
                    "1000"])
    # (0,0): neighbours (1,0),(0,1),(1,1) = 3 live -> dies; (1,0),(0,1),(1,1) likewise
    # (x=3,y=2) is invisible to others; its own visible neighbours are (2,1),(2,2) (+(2,3)? row 3
    # is invisible) -> 0 live -> stays.  (0,3) row 3: neighbours (0,2),(1,2) -> 0 -> stays.
    want = cells_from(["0000",
                       "0000",
                       "0001",
                       "1000"])
    got = O.step_cells(c, O.REF_CLIPPED, O.REF_LITERAL)
    assert (got == want).all(), got
    assert (O.np_step(c, O.REF_CLIPPED, O.REF_LITERAL) == want).all()


def test_clipped_invisible_edge_is_one_way_sink():
    """package.scala:17-28: cells in column w / row h read their neighbours but
    nobody reads them (they are not in [0,w) x [0,h))."""
    w = h = 4
    c = np.zeros((h + 1, w + 1), dtype=np.uint8)
    c[0:3, 4] = 1  # three live cells in the invisible column x = w
    n = O.step_cells(c, O.REF_CLIPPED, O.LIFE)
    assert n[1, 3] == 0  # would be born on a normal board (3 neighbours), but they are invisible
    c2 = np.zeros_like(c)
    c2[0:3, 3] = 1  # visible column x = 3: the invisible cell (4,1) sees 3 -> born
    n2 = O.step_cells(c2, O.REF_CLIPPED, O.LIFE)
    assert n2[1, 4] == 1


def test_blinker_block_glider_torus():
    W = H = 32
    z = np.zeros((H, W), dtype=np.uint8)
    blink = z.copy(); blink[5, 4:7] = 1
    b1 = O.step_cells(blink, O.TORUS, O.LIFE)
    assert b1[4:7, 5].all() and b1.sum() == 3
    assert (O.step_cells(b1, O.TORUS, O.LIFE) == blink).all()
    block = z.copy(); block[10:12, 10:12] = 1
    assert (O.step_cells(block, O.TORUS, O.LIFE) == block).all()
    glider = z.copy()
    for x, y in [(1, 0), (2, 1), (0, 2), (1, 2), (2, 2)]:
        glider[y, x] = 1
    g = glider.copy()
    for _ in range(4):
        g = O.step_cells(g, O.TORUS, O.LIFE)
    assert (g == np.roll(np.roll(glider, 1, 0), 1, 1)).all()
    p, _ = O.run_packed(O.pack(glider), W, 4 * W, O.TORUS, O.LIFE, want_hashes=False)
    assert (O.unpack(p, W) == glider).all()  # full wrap after 4N generations


def test_canonical_words():
    # numpy restatement of the hash's canonical words: column 64k + 2b -> bit b
    # of word 2k, 64k + 2b + 1 -> word 2k + 1; the C oracle's agree
    rng = np.random.default_rng(3)
    for W in (192, 160, 32, 33, 300):
        cells = rng.integers(0, 2, size=(5, W), dtype=np.uint8)
        packed = O.pack(cells)
        dev = O.np_canonical_words(packed, W)
        ww = (W + 31) // 32
        assert dev.shape == (5, ww + (ww % 2))
        for y in range(5):
            for x in range(dev.shape[1] * 32):
                word, bit = 2 * (x // 64) + (x & 1), (x % 64) >> 1
                assert (int(dev[y, word]) >> bit) & 1 == (cells[y, x] if x < W else 0)
            for g in range(dev.shape[1] // 2):
                e, o = ctypes.c_uint32(), ctypes.c_uint32()
                O.lib().oracle_canonical_words(packed[y].ctypes.data_as(O._u32p), ww, g, ctypes.byref(e),
                                               ctypes.byref(o))
                assert (e.value, o.value) == (int(dev[y, 2 * g]), int(dev[y, 2 * g + 1]))


def test_hash_properties():
    for W, topo in [(320, O.TORUS), (352, O.TORUS), (320, O.REF_CLIPPED), (300, O.REF_CLIPPED)]:
        b = O.seed_packed(W, 40, 1)
        assert O.hash_packed(b, W, topology=topo) == O.np_hash(b, W, topology=topo)
    b = O.seed_packed(320, 40, 1)
    h = O.hash_packed(b, 320)
    assert h == O.np_hash(b, 320)
    # a function of the cells alone: the topology (hence the engine's device
    # layout) does not enter it
    assert h == O.hash_packed(b, 320, topology=O.REF_CLIPPED)
    # sharding invariance: partial hashes of row blocks sum to the whole
    parts = [O.hash_packed(b[r0:r1], 320, row0=r0) for r0, r1 in [(0, 7), (7, 30), (30, 40)]]
    assert sum(parts) % (1 << 64) == h
    # every single-bit flip changes it
    rng = np.random.default_rng(0)
    for _ in range(50):
        y, x = int(rng.integers(0, 40)), int(rng.integers(0, 320))
        b2 = b.copy(); b2[y, x // 32] ^= np.uint32(1 << (x % 32))
        assert O.hash_packed(b2, 320) != h
    # the pitch and dead padding words past the width do not enter it
    wide = np.zeros((40, 16), dtype=np.uint32); wide[:, :10] = b
    assert O.hash_packed(wide[:, :10], 320) == h
    # a board W cells wide and the same cells in a wider board (dead columns
    # beyond W) hash alike -- including an odd word count's half group
    b3 = O.seed_packed(96, 8, 5)
    b4 = np.zeros((8, 4), dtype=np.uint32); b4[:, :3] = b3
    assert O.hash_packed(b3, 96) == O.hash_packed(b4, 128) == O.np_hash(b4, 128) == O.np_hash(b3, 96)


def test_hash_keys_odd_and_structured_moves_detected():
    """The keys are odd (a single-word change always changes the hash), and
    the moves Life makes -- a pattern translated by one row or column, or
    two cells of a column moving apart symmetrically (the move a row key
    linear in y could not see) -- change it."""
    for y in (0, 1, 2, 1000, 262143, (1 << 30) - 1):
        assert O.lib().oracle_hash_row_key(y, 0) & 1 and O.lib().oracle_hash_row_key(y, 1) & 1
    for k in (0, 1, 4095, 1 << 20):
        assert O.lib().oracle_hash_pair_key(k) & 1
    W, H = 256, 64
    glider = np.zeros((H, W), dtype=np.uint8)
    for x, y in [(11, 10), (12, 11), (10, 12), (11, 12), (12, 12)]:
        glider[y, x] = 1
    seen = set()
    for dy in range(0, 40):
        for dx in range(0, 70):
            seen.add(O.hash_packed(O.pack(np.roll(np.roll(glider, dy, 0), dx, 1)), W))
    assert len(seen) == 40 * 70
    base = np.zeros((H, W), dtype=np.uint8)
    for d in range(1, 12):
        a = base.copy(); a[30 - d, 77] = a[30 + d, 77] = 1
        b = base.copy(); b[30 - d - 1, 77] = b[30 + d + 1, 77] = 1
        assert O.hash_packed(O.pack(a), W) != O.hash_packed(O.pack(b), W)


def test_seed_sharding_invariant():
    full = O.seed_packed(1000, 50, 9)
    assert (full == O.np_seed(1000, 50, 9)).all()
    assert (O.seed_packed(1000, 50, 9, row0=13, rows=20) == full[13:33]).all()
    assert (full[:, -1] >> np.uint32(1000 % 32) == 0).all()  # padding bits dead


def test_java_random_board_matches_lcg():
    """BoardCreator.scala:23 order: k-th nextBoolean -> (x=k/(h+1), y=k%(h+1))."""
    for seed in (0, 1, 42, -7):
        b = O.java_random_cells(6, 6, seed)
        bools = O.java_random_next_booleans(seed & ((1 << 64) - 1) if seed >= 0 else seed, 49)
        assert all(b[k % 7, k // 7] == bools[k] for k in range(49))
    # External known answers of the JDK LCG: new Random(42).nextInt() is
    # -1170105035 and new Random(0).nextInt() is -1155484576.  nextInt() =
    # next(32) and nextBoolean() = next(1) read the same 48-bit state, so the
    # first nextBoolean() is the sign bit of the first nextInt().
    for seed, first_int in ((42, -1170105035), (0, -1155484576)):
        s = (seed ^ 0x5DEECE66D) & ((1 << 48) - 1)
        s = (s * 0x5DEECE66D + 0xB) & ((1 << 48) - 1)
        v = s >> 16
        signed = v - (1 << 32) if v >= (1 << 31) else v
        assert signed == first_int, (seed, signed)
        assert O.java_random_next_booleans(seed, 1) == [first_int < 0]


def test_golden_ref_default_reproduces():
    for entry in GOLDEN["ref_default"]:
        cells = cells_from(entry["initial"])
        assert (cells == O.java_random_cells(entry["w"], entry["h"], entry["java_seed"])).all()
        for name, res in entry["modes"].items():
            rule = {"life": O.LIFE, "ref-literal": O.REF_LITERAL, "ref-effective": O.REF_EFFECTIVE}[name]
            p, hashes = O.run_packed(O.pack(cells), entry["w"] + 1, 100, O.REF_CLIPPED, rule)
            assert [int(x) for x in hashes] == res["hashes"]
            assert (O.unpack(p, entry["w"] + 1) == cells_from(res["boards"][-1]["cells"])).all()
            if name == "ref-effective":
                assert len(set(res["hashes"])) == 1  # the identity: the board never changes


@pytest.mark.parametrize("idx", [1, 2])
def test_golden_torus_small_reproduces(idx):
    g = GOLDEN["torus"][idx]
    rule = {"life": O.LIFE, "ref-literal": O.REF_LITERAL}[g["rule"]]
    b = O.seed_packed(g["W"], g["H"], g["seed"])
    assert O.hash_packed(b, g["W"]) == g["hash0"]
    _, hashes = O.run_packed(b, g["W"], g["gens"], O.TORUS, rule)
    assert [int(x) for x in hashes] == g["hashes"]


def test_golden_torus_4096_first_generations():
    g = GOLDEN["torus"][0]
    assert (g["W"], g["H"], g["gens"]) == (4096, 4096, 1000)
    b = O.seed_packed(4096, 4096, g["seed"])
    assert O.hash_packed(b, 4096) == g["hash0"]
    _, hashes = O.run_packed(b, 4096, 20, O.TORUS, O.LIFE)
    assert [int(x) for x in hashes] == g["hashes"][:20]


def test_bench_golden_table_epoch0_and_shape():
    """tests/golden/bench_262144.json (bench.py's parity table): epoch 0 is
    the oracle's hash of the seed-0x5EED 262144^2 board, recomputed here in
    row blocks (the hash is a sum over rows, the seed a function of the word
    index); epochs 1..140 come from make_bench_golden.py's oracle run and are
    checked on the GPU (the loopback N = 8 ring, config 5 at full size)."""
    import json
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bench_262144.json")
    with open(path) as f:
        d = json.load(f)
    assert d["board"] == [262144, 262144] and d["seed"] == 0x5EED and d["rule"] == "B3/S23"
    hashes = [int(x, 16) for x in d["hashes"]]
    assert len(hashes) == 141 and len(set(hashes)) == 141
    W = H = 262144
    total, block = 0, 2048
    for r0 in range(0, H, block):
        blk = O.seed_packed(W, H, 0x5EED, row0=r0, rows=block)
        total = (total + O.hash_packed(blk, W, row0=r0)) % (1 << 64)
    assert total == hashes[0]

