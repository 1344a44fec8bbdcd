"""GPU parity: libgol (HIP, gfx950) vs the CPU oracle, through the C ABI.

Bar: bit-exact boards and per-generation state hashes (integer/bit work).
Oracle: oracle/ (parity unpinned -- see oracle/gol_oracle.c header).
"""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))
RULES = {"life": O.LIFE, "ref-literal": O.REF_LITERAL, "ref-effective": O.REF_EFFECTIVE}


def engine(*a, **k):
    from gameoflife.engine import GolEngine
    return GolEngine(*a, **k)


def rule_obj(rule):
    from gameoflife.rules import Rule
    return Rule(rule[0], rule[1])


GPP = [1, 2, 3, 4, 5, 8, 10, 12]  # generations fused per HBM pass (temporal blocking depth)


def check_run(W, H, gens, rule=O.LIFE, topology="torus", seed=None, cells=None, band=0, gpp=1,
              vec=0):
    topo = O.TORUS if topology == "torus" else O.REF_CLIPPED
    if cells is not None:
        board = O.pack(cells)
    else:
        board = O.seed_packed(W, H, seed if seed is not None else 0x5EED)
    with engine(W, H, topology=topology, rule=rule_obj(rule)) as e:
        e.set_tuning(band_rows=band, gens_per_pass=gpp, words_per_lane=vec)
        e.load(board)
        assert e.hash() == O.hash_packed(board, W, topology=topo)
        got = e.step(gens, hashes=True)
        final_gpu = e.snapshot()
        assert e.epoch == gens
    final_cpu, want = O.run_packed(board, W, gens, topo, rule)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"first hash mismatch at generation {bad[0] + 1} ({W}x{H} {topology} {rule})"
    np.testing.assert_array_equal(final_gpu, final_cpu)


def check_run_unhashed_g1(W, H, gens, rule=O.LIFE, topology="torus", seed=0, vec=0, band=0, cells=None):
    """One generation per pass without the fused hash -- step_kernel<VEC, ...,
    HASH=false> with its non-temporal stores, the kernel behind bench.py's
    single_generation_passes line -- checked by the final board word for word
    and gol_hash against the oracle's last per-generation hash."""
    topo = O.TORUS if topology == "torus" else O.REF_CLIPPED
    board = O.pack(cells) if cells is not None else O.seed_packed(W, H, seed)
    with engine(W, H, topology=topology, rule=rule_obj(rule)) as e:
        e.set_tuning(band_rows=band, gens_per_pass=1, words_per_lane=vec)
        assert e.pass_plan(gens) == [1] * gens
        e.load(board)
        e.step(gens)
        h = e.hash()
        final_gpu = e.snapshot()
    final_cpu, want = O.run_packed(board, W, gens, topo, rule)
    np.testing.assert_array_equal(final_gpu, final_cpu)
    assert h == int(want[-1])


def test_selftest_cross_lane(gpu):
    from gameoflife.engine import selftest
    rep = selftest(gpu)
    inp = np.array([(0x01000193 * (i + 1) ^ (i << 24)) & 0xFFFFFFFF for i in range(64)],
                   dtype=np.uint64).astype(np.uint32)
    shr = np.concatenate([[0xA0A0A0A0], inp[:-1]]).astype(np.uint32)
    shl = np.concatenate([inp[1:], [0xB0B0B0B0]]).astype(np.uint32)
    np.testing.assert_array_equal(rep[0:64], shr)
    np.testing.assert_array_equal(rep[64:128], shl)
    prev = np.roll(inp, 1)
    align = ((inp.astype(np.uint64) << 1) | (prev.astype(np.uint64) >> 31)) & 0xFFFFFFFF
    np.testing.assert_array_equal(rep[128:192], align.astype(np.uint32))
    assert (rep[192:256] == inp[5]).all()


def test_seed_matches_oracle(gpu):
    for W, H in [(4096, 64), (100, 7), (32 * 300, 33)]:
        topo = "torus" if W % 32 == 0 else "ref-clipped"
        with engine(W, H, topology=topo) as e:
            e.seed(0x5EED)
            np.testing.assert_array_equal(e.snapshot(), O.seed_packed(W, H, 0x5EED))
            assert e.hash() == O.hash_packed(O.seed_packed(W, H, 0x5EED), W,
                                             topology=O.TORUS if topo == "torus" else O.REF_CLIPPED)


# words per row covering VEC=1/2/4, partial strips, single word, many strips
TORUS_SHAPES = [(32, 8), (64, 3), (96, 17), (32 * 63, 5), (32 * 64, 9), (32 * 128, 40),
                (32 * 130, 11), (32 * 256, 33), (32 * 260, 7), (32 * 1024, 70), (32 * 2048, 4)]


@pytest.mark.parametrize("gpp", GPP)
@pytest.mark.parametrize("W,H", TORUS_SHAPES)
def test_torus_life(gpu, W, H, gpp):
    check_run(W, H, 12, O.LIFE, "torus", seed=W * 7 + H, gpp=gpp)


@pytest.mark.parametrize("gpp", GPP)
@pytest.mark.parametrize("H", [1, 2, 3])
def test_torus_tiny_heights(gpu, H, gpp):
    # rows alias on a torus shorter than 3 rows (multiset count)
    check_run(32 * 8, H, 6, O.LIFE, "torus", seed=H, gpp=gpp)
    check_run(32 * 8, H, 6, (0x1A4, 0x03B), "torus", seed=H, gpp=gpp)


@pytest.mark.parametrize("gpp", GPP)
@pytest.mark.parametrize("band", [1, 2, 3, 5, 7, 16, 1000])
def test_band_sizes(gpu, band, gpp):
    # short bands exercise the boustrophedon direction switch and ring tails
    check_run(32 * 256, 61, 7, O.LIFE, "torus", seed=band, band=band, gpp=gpp)
    check_run(32 * 4, 23, 7, (0x049, 0x16E), "torus", seed=band, band=band, gpp=gpp)


@pytest.mark.parametrize("gpp", GPP)
@pytest.mark.parametrize("seed", range(6))
def test_torus_random_rules(gpu, seed, gpp):
    rng = np.random.default_rng(seed)
    rule = (int(rng.integers(0, 512)), int(rng.integers(0, 512)))
    W = 32 * int(rng.choice([1, 3, 64, 130, 256, 300]))
    H = int(rng.integers(1, 50))
    check_run(W, H, 8, rule, "torus", seed=seed, gpp=gpp)


@pytest.mark.parametrize("gpp", GPP)
@pytest.mark.parametrize("name", list(RULES))
def test_torus_named_rules(gpu, name, gpp):
    check_run(32 * 96, 31, 10, RULES[name], "torus", seed=3, gpp=gpp)


@pytest.mark.parametrize("gpp", [1, 2, 3, 4, 6, 7, 8, 9, 11, 12])
@pytest.mark.parametrize("vec", [1, 2, 4])
def test_words_per_lane(gpu, vec, gpp):
    # every lane width at every depth, full and partial strips, torus and clipped
    check_run(32 * 520, 37, 9, O.LIFE, "torus", seed=vec, gpp=gpp, vec=vec)
    rng = np.random.default_rng(vec * 10 + gpp)
    cells = (rng.random((31, 32 * 132 - 9)) < 0.5).astype(np.uint8)
    if vec == 4 and gpp > 7:
        # the 16-byte-lane generic-rule / clipped instances deeper than 7
        # would spill to scratch: gol_set_tuning refuses them
        from gameoflife import _native as N
        for W, topo in ((32 * 12, "torus"), (32 * 132 - 9, "ref-clipped")):
            with engine(W, 29, topology=topo, rule=rule_obj((0x0C8, 0x1A6))) as e:
                with pytest.raises(N.GolError) as ei:
                    e.set_tuning(gens_per_pass=gpp, words_per_lane=vec)
                assert ei.value.code == N.GOL_EINVAL
        return
    check_run(32 * 12, 29, 9, (0x0C8, 0x1A6), "torus", seed=vec, gpp=gpp, vec=vec)
    check_run(32 * 132 - 9, 31, 9, O.LIFE, "ref-clipped", cells=cells, gpp=gpp, vec=vec)


def test_words_per_lane_4_planner_caps_generic_depth(gpu):
    # 16-byte lanes forced with automatic depth: the planner keeps the generic
    # and clipped instances at <= 7 generations per pass (no scratch spills)
    with engine(32 * 12, 29, topology="torus", rule=rule_obj((0x0C8, 0x1A6))) as e:
        e.set_tuning(words_per_lane=4)
        assert max(e.pass_plan(60)) <= 7 and max(e.pass_plan(60, hashes=True)) <= 7
    check_run(32 * 132 - 9, 31, 20, O.LIFE, "ref-clipped",
              cells=(np.random.default_rng(5).random((31, 32 * 132 - 9)) < 0.5).astype(np.uint8), gpp=0, vec=4)


@pytest.mark.parametrize("vec", [1, 2, 4])
@pytest.mark.parametrize("W,H", TORUS_SHAPES)
def test_unhashed_single_generation_torus(gpu, W, H, vec):
    # every lane width; full and partial strips (e.g. 130 words = 2 strips of
    # 64 x 2 words, the second with one lane), a single word, many strips
    if (W // 32) % vec:
        pytest.skip("words per lane must divide the row")
    check_run_unhashed_g1(W, H, 5, seed=W + H + vec, vec=vec)


@pytest.mark.parametrize("band", [1, 3, 4, 6, 8, 16, 0])  # 4 / 6 / 8: step_kernel's straight-line band paths
def test_unhashed_single_generation_bands_rules_clipped(gpu, band):
    check_run_unhashed_g1(32 * 520, 37, 4, seed=band, band=band)
    check_run_unhashed_g1(32 * 12, 29, 4, rule=(0x0C8, 0x1A6), seed=band, band=band)
    rng = np.random.default_rng(band)
    cells = (rng.random((31, 32 * 132 - 9)) < 0.5).astype(np.uint8)
    check_run_unhashed_g1(32 * 132 - 9, 31, 4, topology="ref-clipped", cells=cells, band=band)


def test_tuning_rejects_bad_values(gpu):
    from gameoflife import _native as N
    with engine(32 * 6, 8) as e:
        for kw in [dict(gens_per_pass=13), dict(words_per_lane=3), dict(words_per_lane=4),
                   dict(band_rows=-1)]:
            with pytest.raises(N.GolError):
                e.set_tuning(**kw)


@pytest.mark.parametrize("gpp", GPP)
def test_gens_not_multiple_of_depth(gpu, gpp):
    # remainder passes run at a shallower depth; hashes stay per generation
    for gens in (1, 5, 7, 13):
        check_run(32 * 300, 45, gens, O.LIFE, "torus", seed=gens, gpp=gpp)


# (2, 2) and one-cell-wide boards are refused (tests/test_degenerate_geometry.py)
CLIPPED_SHAPES = [(7, 7), (2, 3), (3, 2), (33, 40), (100, 65), (32, 9), (1000, 37), (32 * 300 + 5, 12),
                  (64 * 32 + 1, 20)]


@pytest.mark.parametrize("gpp", GPP)
@pytest.mark.parametrize("W,H", CLIPPED_SHAPES)
@pytest.mark.parametrize("name", list(RULES))
def test_ref_clipped(gpu, W, H, name, gpp):
    rng = np.random.default_rng(W * 31 + H)
    cells = (rng.random((H, W)) < 0.45).astype(np.uint8)
    check_run(W, H, 6, RULES[name], "ref-clipped", cells=cells, gpp=gpp)


@pytest.mark.parametrize("gpp", GPP)
def test_ref_clipped_random_rules(gpu, gpp):
    rng = np.random.default_rng(99)
    for _ in range(6):
        rule = (int(rng.integers(0, 512)), int(rng.integers(0, 512)))
        W, H = int(rng.integers(2, 400)), int(rng.integers(2, 60))
        if W == H == 2:
            continue  # refused: the reference stalls (tests/test_degenerate_geometry.py)
        cells = (rng.random((H, W)) < 0.5).astype(np.uint8)
        check_run(W, H, 5, rule, "ref-clipped", cells=cells, gpp=gpp)


def test_golden_ref_default_board(gpu):
    """BASELINE.json config 1 geometry: the reference's default 6x6 board =
    7x7 cells, java.util.Random-seeded, 100 generations, all three rules."""
    for entry in GOLDEN["ref_default"]:
        w, h = entry["w"], entry["h"]
        cells = np.array([[int(ch) for ch in row] for row in entry["initial"]], dtype=np.uint8)
        assert (cells == O.java_random_cells(w, h, entry["java_seed"])).all()
        for name, res in entry["modes"].items():
            for gpp in GPP:
                with engine(w + 1, h + 1, topology="ref-clipped", rule=name) as e:
                    e.set_tuning(gens_per_pass=gpp)
                    e.load(O.pack(cells))
                    got = e.step(100, hashes=True)
                    assert [int(x) for x in got] == res["hashes"], (entry["java_seed"], name, gpp)
                    final = O.unpack(e.snapshot(), w + 1)
                    want = np.array([[int(ch) for ch in row] for row in res["boards"][-1]["cells"]])
                    assert (final == want).all()


@pytest.mark.parametrize("gpp", GPP)
def test_golden_torus_4096_1000(gpu, gpp):
    """BASELINE.json config 2: 4096^2 torus B3/S23, 1000 generations,
    per-generation hashes bit-exact against the committed oracle vectors."""
    for g in GOLDEN["torus"]:
        with engine(g["W"], g["H"], topology="torus", rule=g["rule"]) as e:
            e.set_tuning(gens_per_pass=gpp)
            e.seed(g["seed"])
            assert e.hash() == g["hash0"]
            got = e.step(g["gens"], hashes=True)
            bad = np.nonzero(got != np.array(g["hashes"], dtype=np.uint64))[0]
            assert bad.size == 0, f"{g['W']}x{g['H']}: first mismatch at generation {bad[0] + 1}"
            assert e.hash() == g["final_hash"]


def test_fused_hash_equals_standalone_hash(gpu):
    with engine(32 * 512, 300) as e:
        e.seed(5)
        for _ in range(4):
            h = e.step(1, hashes=True)[0]
            assert h == e.hash()


@pytest.mark.parametrize("W", [32 * 130, 32 * 129, 32 * 2, 32])
def test_hash_is_a_function_of_the_cells(gpu, W):
    """The state hash reads the cells through canonical words (DESIGN.md
    section 5): the same cells held by a pair-layout torus (even word count),
    a row-major torus (odd word count) and a row-major clipped board hash
    alike -- gol_hash and the fused per-generation hashes of the identity
    rule, which keeps the board -- and equal the oracle's value."""
    from gameoflife import _native as N
    rng = np.random.default_rng(W)
    cells = (rng.random((23, W)) < 0.5).astype(np.uint8)
    board = O.pack(cells)
    want = O.hash_packed(board, W)
    got = {}
    for topo in ("torus", "ref-clipped"):
        with engine(W, 23, topology=topo, rule=rule_obj(O.REF_EFFECTIVE)) as e:
            e.load(board)
            got[topo] = (e.hash(), [int(x) for x in e.step(3, hashes=True)])
    assert got["torus"] == got["ref-clipped"] == (want, [want] * 3)
    assert N.device_layout(W) == (2 if (W // 32) % 2 == 0 else 1) and N.device_layout(W, N.GOL_REF_CLIPPED) == 1


def test_snapshot_get_cell_checkpoint(gpu):
    W, H = 32 * 70, 50
    with engine(W, H) as e:
        e.seed(9)
        e.step(7)
        snap = e.snapshot()
        cells = O.unpack(snap, W)
        for (x, y) in [(0, 0), (W - 1, H - 1), (123, 17), (31, 32), (32, 1)]:
            assert e.get_cell(x, y) == bool(cells[y, x])
        blob = e.checkpoint()
        ref = e.step(5, hashes=True)
        e.restore(blob)
        assert e.epoch == 7
        np.testing.assert_array_equal(e.snapshot(), snap)
        np.testing.assert_array_equal(e.step(5, hashes=True), ref)


@pytest.mark.parametrize("W", [32 * 70, 32 * 71])  # pair-interleaved / row-major device words
def test_get_cell_every_layout(gpu, W):
    H = 37
    rng = np.random.default_rng(W)
    with engine(W, H) as e:
        e.seed(11)
        e.step(13)  # default pass depth (6) plus a remainder pass
        cells = O.unpack(e.snapshot(), W)
        for _ in range(200):
            x, y = int(rng.integers(0, W)), int(rng.integers(0, H))
            assert e.get_cell(x, y) == bool(cells[y, x]), (x, y)
        for x in (0, 1, 31, 32, 63, 64, 65, W - 2, W - 1):
            assert e.get_cell(x, 5) == bool(cells[5, x]), x


def test_full_size_65536_bit_exact(gpu):
    """BASELINE.json config 3 geometry (65536^2 torus): 6 generations checked
    word-for-word against the multithreaded CPU oracle, including one pass of
    the automatic depth (6) the benchmark runs."""
    W = H = 65536
    board = O.seed_packed(W, H, 0x5EED)
    final_cpu, want = O.run_packed(board, W, 6, O.TORUS, O.LIFE)
    for gpp in (1, 2, 4, 0):
        with engine(W, H) as e:
            e.set_tuning(gens_per_pass=gpp)
            e.seed(0x5EED)
            got = e.step(6, hashes=True)
            final = e.snapshot()
        np.testing.assert_array_equal(got, want)
        assert (final == final_cpu).all(), gpp
    with engine(W, H) as e:  # the benchmark's own path: no fused hash
        e.seed(0x5EED)
        e.step(6)
        assert (e.snapshot() == final_cpu).all()


def test_known_patterns_on_gpu(gpu):
    # glider on a 64x64 torus returns to its start after 4*64 generations
    W = H = 64
    cells = np.zeros((H, W), dtype=np.uint8)
    for x, y in [(1, 0), (2, 1), (0, 2), (1, 2), (2, 2)]:
        cells[y, x] = 1
    with engine(W, H) as e:
        e.load(O.pack(cells))
        e.step(4)
        shifted = np.roll(np.roll(cells, 1, 0), 1, 1)
        assert (O.unpack(e.snapshot(), W) == shifted).all()
        e.step(4 * 64 - 4)
        assert (O.unpack(e.snapshot(), W) == cells).all()


def test_pass_plan(gpu):
    """gol_pass_plan: the depths cover the generations exactly, respect the
    cap (12 on the B3/S23 torus, 8 for other rules and the clipped topology,
    or a fixed gens_per_pass), run deepest first, and follow the cost table
    (DESIGN.md "Pass planner")."""
    with engine(32 * 300, 64) as e:  # narrow (3 strips): 10-generation passes (round-4 paired kernels)
        for n in (1, 5, 6, 7, 13, 50, 60, 1024):
            plan = e.pass_plan(n)
            assert sum(plan) == n and all(1 <= g <= 12 for g in plan), (n, plan)
            assert plan == sorted(plan, reverse=True), plan
        assert e.pass_plan(48) == [10] * 3 + [9] * 2
        assert e.pass_plan(102) == [10] * 7 + [9, 9, 7, 7]
        assert e.pass_plan(60, hashes=True) == [10] * 6
        e.set_tuning(gens_per_pass=4)
        assert e.pass_plan(10) == [4, 4, 2]
    with engine(262144, 64) as e:  # wide (67 strips): G = 10, the deepest paired kernel at 3 waves/SIMD
        assert e.pass_plan(60) == [10] * 6
        assert e.pass_plan(20) == [10, 10]
        assert e.pass_plan(12) == [12]
        assert e.pass_plan(60, hashes=True) == [10] * 6
        assert e.pass_plan(20, hashes=True) == [10, 10]
        check = e.pass_plan(13)
        assert sum(check) == 13
    with engine(262144, 64, rule=rule_obj(O.REF_EFFECTIVE)) as e:  # other rules: planned passes stop at 8
        assert max(e.pass_plan(60)) <= 8 and sum(e.pass_plan(60)) == 60
    with engine(4096, 4096) as e:  # small board (configs[1]): hashed passes plan like unhashed ones
        assert e.pass_plan(1000, hashes=True) == [10] * 100 == e.pass_plan(1000)
    with engine(65536, 65536) as e:  # fills the GPU: the hashed narrow row's G = 7 tie stands
        assert 7 in e.pass_plan(1000, hashes=True)


def test_snapshot_into_caller_buffer(gpu):
    """gol_snapshot into a caller-owned buffer (GolEngine.snapshot(out=...)):
    same board as a fresh snapshot; a buffer of the wrong shape or dtype is
    refused before the copy."""
    W, H = 4096, 77
    board = O.seed_packed(W, H, 5)
    with engine(W, H, topology="torus", rule=rule_obj(O.LIFE)) as e:
        e.load(board)
        e.step(3)
        fresh = e.snapshot()
        buf = np.full(fresh.shape, 0xFFFFFFFF, dtype=np.uint32)
        assert e.snapshot(out=buf) is buf
        np.testing.assert_array_equal(buf, fresh)
        np.testing.assert_array_equal(fresh, O.run_packed(board, W, 3)[0])
        for bad in (np.zeros((H, W // 32 + 1), np.uint32), np.zeros((H, W // 32), np.int64),
                    np.zeros((W // 32, H), np.uint32).T):
            with pytest.raises(ValueError):
                e.snapshot(out=bad)


def test_step_ex_checks_hash_capacity(gpu):
    """gol_step_ex refuses a hashes_out buffer shorter than the generations
    asked for, before advancing anything (the JVM worker passes its direct
    buffer's capacity)."""
    import ctypes

    from gameoflife import _native as N
    with engine(32 * 64, 40) as e:
        e.seed(3)
        buf = np.zeros(4, dtype=np.uint64)
        rc = N.lib.gol_step_ex(e._h, 5, buf.ctypes.data_as(N._u64p), buf.size)
        assert rc == N.GOL_EINVAL and e.epoch == 0
        assert N.lib.gol_step_ex(e._h, 4, buf.ctypes.data_as(N._u64p), buf.size) == N.GOL_OK
        assert e.epoch == 4 and buf[-1] == e.hash()
        assert N.lib.gol_step_ex(e._h, 3, ctypes.cast(None, N._u64p), 0) == N.GOL_OK
        assert e.epoch == 7


@pytest.mark.parametrize("W,topology", [(32 * 70, "torus"), (32 * 71, "torus"), (32 * 40 + 5, "ref-clipped")])
@pytest.mark.parametrize("row0,rows,d", [(10, 9, 4), (0, 12, 7), (30, 10, 13), (0, 40, 3)])
def test_replay_light_cone(gpu, W, topology, row0, rows, d):
    """gol_replay: a shard restored at epoch e, given the d rows above and
    below it at epoch e (wrapping on a torus, dead beyond a clipped edge),
    advances d generations alone exactly as the whole board does; its
    per-generation partial hashes are the whole board's rows' hashes."""
    from gameoflife.elastic import light_cone_from
    H = 40
    topo = O.TORUS if topology == "torus" else O.REF_CLIPPED
    board = O.seed_packed(W, H, row0 * 7 + d)
    with engine(W, H, topology=topology, rule=rule_obj(O.LIFE), row0=row0, rows=rows) as e:
        e.load(board[row0:row0 + rows])
        up, dn = light_cone_from(lambda idx: board[idx], row0, rows, d, H, topology == "torus", e.wwords)
        got = e.replay(d, up, dn)
        assert e.epoch == d
        cur = board
        for g in range(d):
            cur, _ = O.run_packed(cur, W, 1, topo, O.LIFE, want_hashes=False)
            assert got[g] == O.hash_packed(cur[row0:row0 + rows], W, row0=row0, topology=topo), g
        assert (e.snapshot() == cur[row0:row0 + rows]).all()
        with pytest.raises(Exception):
            e.replay(2, up[:1], dn[:1])  # light-cone rows of the wrong depth


def test_profile_clock_probe(gpu):
    """gol_profile_clock: the in-kernel probe (every workgroup's XCD core-clock
    and 100 MHz reference counters at start and end) yields the clock of the
    profiled launches -- plausible for an MI355X (its max is 2.4 GHz) -- and
    the probe leaves the results bit-exact."""
    W, H = 32 * 1024, 1024
    board = O.seed_packed(W, H, 0x5EED)
    with engine(W, H) as e:
        e.seed(0x5EED)
        e.profile(True)
        e.profile_reset()
        assert e.profile_clock() == 0.0
        got = e.step(40, hashes=True)
        ms, n, g = e.profile_read()
        clk = e.profile_clock()
        assert n > 0 and g == 40 and 0.3 < clk < 2.6, clk
        e.profile_reset()
        assert e.profile_clock() == 0.0
        e.profile(False)
        final = e.snapshot()
    want_board, want = O.run_packed(board, W, 40)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(final, want_board)
