"""GPU: boards at the edges of the geometry the kernels index, against the CPU
oracle (bit-exact boards and every generation's hash).

* very wide tori: 2^24 columns (524288 words: 4229 column strips of the
  multi-generation kernels, 8192 of the single-generation one) -- the strip
  and column arithmetic far past the bench's 262144 columns;
* very tall narrow tori: 2^20 rows of one pair (64 columns: a single strip
  whose halo lanes wrap onto the same pair), and of one word (32 columns,
  row-major);
* a clipped board of 2^20 + 5 columns (a partial last word) and 40 rows;
* the small-board band rule's smallest bands (gol_schedule.cpp
  small_board_band) on tori of 1 and 2 strips, at every depth the planner
  picks and a few fixed ones;
* whole-row waves (gol_kernels.h whole_row_fits: a 4096-column B3/S23 torus
  at 10-generation passes runs one 64-lane strip whose row wraps by wave
  rotates): square and odd-height boards, fixed bands from 1 row to more than
  the board, hashed and not, and as a 1-rank RCCL self-ring (interior and
  boundary launches);
* the tail split (gol_schedule.cpp tail_split: the last round of resident
  waves in bands of band / 6 below 768-row bands) on boards of an odd row
  count, so the bulk range ends in a partial band before the tail bands.
The planner chooses the depths unless a test fixes them."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _run(W, H, gens, topology="torus", gpp=0, seed=0x5EED):
    from gameoflife.engine import GolEngine
    topo = O.TORUS if topology == "torus" else O.REF_CLIPPED
    if topology == "torus":
        board = O.seed_packed(W, H, seed)
    else:
        rng = np.random.default_rng(seed)
        board = O.pack((rng.random((H, W)) < 0.5).astype(np.uint8))
    with GolEngine(W, H, topology=topology, rule="life") as e:
        e.set_tuning(gens_per_pass=gpp)
        e.load(board)
        got = e.step(gens, hashes=True)
        final_gpu = e.snapshot()
        plan = e.pass_plan(gens, hashes=True)
    final_cpu, want = O.run_packed(board, W, gens, topo, O.LIFE, nthreads=0)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{W}x{H} {topology}: first hash mismatch at generation {bad[0] + 1}, plan {plan}"
    np.testing.assert_array_equal(final_gpu, final_cpu)
    return plan


@pytest.mark.parametrize("gpp", [0, 1, 7])
def test_very_wide_torus(gpu, gpp):
    plan = _run(1 << 24, 40, 14, gpp=gpp)
    assert not gpp or max(plan) == gpp


@pytest.mark.parametrize("W", [64, 32])
def test_very_tall_narrow_torus(gpu, W):
    _run(W, 1 << 20, 24)


def test_wide_clipped_board_with_partial_word(gpu):
    _run((1 << 20) + 5, 40, 12, topology="ref-clipped")


@pytest.mark.parametrize("S", [1024, 2048, 3968, 4096, 8192])
@pytest.mark.parametrize("gpp", [0, 4, 12])
def test_small_board_bands(gpu, S, gpp):
    """3968 columns = 62 pairs: exactly one strip; 4096 = 62 + 2 pairs."""
    _run(S, S // 4, 26, gpp=gpp, seed=S + gpp)


@pytest.mark.parametrize("W,H", [(131072, 30001), (65536, 65535)])
def test_tail_split_odd_rows(gpu, W, H):
    """34 strips x 118 256-row bands and 17 x 256: both more than one round of
    resident waves, so the planned 10-generation passes end in tail bands."""
    _run(W, H, 20, seed=H)


@pytest.mark.parametrize("H,band", [(4096, 0), (4096, 1), (4096, 7), (4097, 4), (333, 0), (20, 0), (4096, 5000)])
def test_whole_row_waves(gpu, H, band):
    """4096 columns = 128 words = one wave of pairs: every 10-generation pass
    runs the whole-row instance (the plan is all 10s), against the oracle."""
    from gameoflife.engine import GolEngine
    W, gens = 4096, 30
    board = O.seed_packed(W, H, H + band)
    for hashed in (False, True):
        with GolEngine(W, H, topology="torus", rule="life") as e:
            e.set_tuning(band_rows=band, gens_per_pass=10)
            e.load(board)
            got = e.step(gens, hashes=hashed)
            final_gpu = e.snapshot()
        final_cpu, want = O.run_packed(board, W, gens, O.TORUS, O.LIFE, nthreads=0)
        np.testing.assert_array_equal(final_gpu, final_cpu)
        if hashed:
            bad = np.nonzero(got != want)[0]
            assert bad.size == 0, f"first hash mismatch at generation {bad[0] + 1}"


def test_whole_row_waves_self_ring(gpu):
    """The same board as a 1-rank RCCL self-ring: the sharded pass's interior
    rows and its two boundary row blocks (two row ranges in one launch) both
    run whole-row waves."""
    from gameoflife import _native as N
    from gameoflife.engine import GolEngine
    W, H, gens = 4096, 512, 40
    board = O.seed_packed(W, H, 77)
    with GolEngine(W, H, topology="torus", rule="life") as e:
        e.comm_init(N.unique_id(), 0, 1)
        e.load(board)
        got = e.step(gens, hashes=True)
        final_gpu = e.snapshot()
    final_cpu, want = O.run_packed(board, W, gens, O.TORUS, O.LIFE, nthreads=0)
    np.testing.assert_array_equal(final_gpu, final_cpu)
    assert (got == want).all()
