"""GPU parity of the unhashed multi-generation passes at every depth.

tests/test_gpu_parity.py steps with the fused hash (its check_run compares
per-generation hashes), so most multi-generation checks there run the
hashed kernel instances; the benchmark's headline passes are the UNHASHED
instances of multistep_hg_kernel.  Every check here steps without hashes
and compares the final board word for word and gol_hash with the CPU
oracle: every depth G = 2..12 (one kernel instance each) on rows of 1 to 67
column strips (124 words per strip: rows of exactly k * 124 words and either
side of them, tori narrower than one wave, whose lanes wrap the row several
times), band heights, generic rules, the 262144-column row of the benchmark
and the sharded schedule (in-process group).  The same file checked the
shared edge lanes A/B'd in round 3 (DESIGN.md §4 "Tall bands", last
paragraph).  Oracle: oracle/ (parity unpinned -- see oracle/gol_oracle.c
header)."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

# words per row: one pair / two pairs; under one wave; 62 / 63 / 64 pairs; exact
# multiples of the 124-word pair strip and of 248 (and of 126) and either side
# of them; many strips.
WORDS = [2, 4, 60, 122, 124, 126, 128, 244, 246, 248, 250, 252, 254, 372, 378, 380, 492, 496, 500, 1024, 8190, 8192]
DEPTHS = list(range(2, 13))


def engine(*a, **k):
    from gameoflife.engine import GolEngine
    return GolEngine(*a, **k)


def rule_obj(rule):
    from gameoflife.rules import Rule
    return Rule(rule[0], rule[1])


def check_unhashed(W, H, gens, gpp, rule=O.LIFE, seed=0, band=0):
    board = O.seed_packed(W, H, seed)
    with engine(W, H, topology="torus", rule=rule_obj(rule)) as e:
        e.set_tuning(band_rows=band, gens_per_pass=gpp)
        e.load(board)
        e.step(gens)
        h = e.hash()
        final_gpu = e.snapshot()
    final_cpu, want = O.run_packed(board, W, gens, O.TORUS, rule)
    bad = np.argwhere(final_gpu != final_cpu)
    assert bad.size == 0, f"{W}x{H} G={gpp}: first wrong word (row, col) {tuple(bad[0])}"
    assert h == int(want[-1])


def test_strip_geometry(gpu):
    """gol_occupancy reports 124-word strips (62 output lanes x 2 words) for
    multi-generation passes on the pair layout, 128 or 256 (64 lanes) for
    single-generation passes, 62 (one word per lane) where the layout is
    row-major (odd word count) and 128 for the whole-row waves of a
    4096-column torus."""
    for words in (8192, 8190):
        with engine(32 * words, 16) as e:
            for g in DEPTHS:
                assert e.occupancy(g)[1] == 124, (words, g)
            assert e.occupancy(1)[1] in (128, 256)
    with engine(32 * 8191, 16) as e:  # odd word count: row-major words
        assert e.occupancy(12)[1] == 62
    with engine(4096, 16) as e:  # one wave of pairs per row: whole-row waves at G = 10 only
        assert e.occupancy(10)[1] == 128 and e.occupancy(9)[1] == 124


def test_headline_instance_keeps_three_waves(gpu):
    """The planner's headline depth on wide B3/S23 tori (G = 10, the
    row-pair-shared circuit) holds 3 waves per SIMD
    (12 per CU): at 163 VGPRs it sits 5 below the 3-wave limit, and a change
    that crosses it (G = 11 / 12 already run at 2) must show here rather than
    only as a slower bench."""
    with engine(262144, 64) as e:
        assert e.pass_plan(20) == [10, 10]
        assert e.occupancy(10)[0] >= 12
        assert e.occupancy(8)[0] >= 12


@pytest.mark.parametrize("gpp", DEPTHS)
@pytest.mark.parametrize("words", WORDS)
def test_unhashed_every_depth(gpu, words, gpp):
    H = 2 * gpp + 7  # rows < a band and > 2G: every stream row of a band wraps once
    check_unhashed(32 * words, H, 2 * gpp + 1, gpp, seed=words * 13 + gpp)


@pytest.mark.parametrize("gpp", [2, 7, 12])
@pytest.mark.parametrize("band", [1, 3, 16, 1000])
def test_unhashed_bands(gpu, band, gpp):
    # short bands: the boustrophedon direction switch and ring tails
    check_unhashed(32 * 254, 61, 2 * gpp, gpp, seed=band, band=band)


@pytest.mark.parametrize("gpp", [3, 8, 12])
@pytest.mark.parametrize("rule", [(0x049, 0x16E), O.REF_EFFECTIVE, O.REF_LITERAL])
def test_unhashed_generic_rules(gpu, rule, gpp):
    # the generic-rule instances of the horizontal-first kernel
    check_unhashed(32 * 380, 29, gpp + 3, gpp, rule=rule, seed=gpp)


def test_unhashed_wide_row(gpu):
    """262144 columns (66 strips of 124 words and one of 32 words): the
    planner's own passes for 20 generations (the bench's kernel instances;
    tests/test_gpu_fullsize.py runs them over the bench's band schedule)."""
    check_unhashed(262144, 1024, 20, 0, seed=0x5EED)


@pytest.mark.parametrize("n", [2, 3])
@pytest.mark.parametrize("gpp", [2, 12])
def test_unhashed_group(gpu, n, gpp):
    """The sharded schedule (interior launch + boundary rows), unhashed: an
    in-process group of row shards."""
    from gameoflife.engine import ShardGroup
    from gameoflife.shard import shard_rows_py
    W, H, gens = 32 * 252, 83, 2 * gpp + 1
    full = O.seed_packed(W, H, 21 + n)
    shards = []
    for k in range(n):
        r0, rows = shard_rows_py(H, k, n)
        e = engine(W, H, row0=r0, rows=rows)
        e.set_tuning(gens_per_pass=gpp)
        e.load(full[r0:r0 + rows])
        shards.append(e)
    g = ShardGroup(shards)
    g.step(gens)
    board = g.snapshot()
    g.close()
    for s in shards:
        s.close()
    ref, _ = O.run_packed(full, W, gens, O.TORUS, O.LIFE, want_hashes=False)
    assert (board == ref).all()


@pytest.mark.parametrize("gpp", [2, 5, 8])
@pytest.mark.parametrize("W", [7, 100, 32 * 62 + 5, 32 * 130 - 9, 32 * 300 + 17])
@pytest.mark.parametrize("rule", [O.REF_EFFECTIVE, O.REF_LITERAL, O.LIFE])
def test_unhashed_clipped(gpu, W, gpp, rule):
    """The reference geometry (ref-clipped, row-major words, any width) without
    the fused hash: the unhashed clipped instances switch off the lanes past
    their last strip's halo lane too (GOL_IDLE_LANES_OFF)."""
    H = 23
    rng = np.random.default_rng(W * 3 + gpp)
    cells = (rng.random((H, W)) < 0.5).astype(np.uint8)
    board = O.pack(cells)
    with engine(W, H, topology="ref-clipped", rule=rule_obj(rule)) as e:
        e.set_tuning(gens_per_pass=gpp)
        e.load(board)
        e.step(2 * gpp + 1)
        h = e.hash()
        final_gpu = e.snapshot()
    final_cpu, want = O.run_packed(board, W, 2 * gpp + 1, O.REF_CLIPPED, rule)
    np.testing.assert_array_equal(final_gpu, final_cpu)
    assert h == int(want[-1])
