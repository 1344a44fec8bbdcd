"""The reference's degenerate boards.

On a ref-clipped board where some cell has no visible neighbour the reference
never completes a generation: that cell's gatherer has nobody to ask, so it
never commits epoch 1 (NextStateCellGathererActor.scala:26-27,39-58,
CellActor.scala:92-94) and its neighbours' requests for that epoch queue
forever (CellActor.scala:75-76).  libgol refuses those boards in gol_create
(GOL_EINVAL) instead of advancing them with results the reference never
produces.  The set of refused boards is pinned against
oracle.reference_commit_epochs, a restatement of the reference's commit
condition.  gol_create validates the geometry before it looks for a device,
so this runs on CPU (accepted boards then fail with GOL_ENODEV) and on the
GPU box (they are created)."""
import pytest

from oracle import oracle as O


def _create(W, H, **kw):
    from gameoflife import _native as N
    from gameoflife.engine import GolEngine
    try:
        GolEngine(W, H, topology="ref-clipped", rule="life", **kw).close()
        return N.GOL_OK
    except N.GolError as e:
        return e.code


def test_commit_condition_restatement():
    # w = h = 1: cell (0,0) has no visible neighbour and stays at epoch 0; the
    # other three commit epoch 1 from its epoch-0 answer and stop there
    ep = O.reference_commit_epochs(1, 1, 10)
    assert ep == {(0, 0): 0, (0, 1): 1, (1, 0): 1, (1, 1): 1}
    # w = 0 or h = 0: nobody has a visible neighbour
    assert set(O.reference_commit_epochs(0, 4, 10).values()) == {0}
    assert set(O.reference_commit_epochs(3, 0, 10).values()) == {0}
    # every other board advances as far as it is driven
    assert set(O.reference_commit_epochs(6, 6, 10).values()) == {10}  # the default board (application.conf:32-33)
    assert set(O.reference_commit_epochs(1, 2, 7).values()) == {7}


@pytest.mark.parametrize("w", range(0, 5))
@pytest.mark.parametrize("h", range(0, 5))
def test_gol_create_refuses_exactly_the_stalling_boards(w, h):
    from gameoflife import _native as N
    rc = _create(w + 1, h + 1)
    if O.reference_completes(w, h):
        assert rc in (N.GOL_OK, N.GOL_ENODEV), rc
    else:
        assert rc == N.GOL_EINVAL


def test_refusal_message_cites_the_reference():
    from gameoflife import _native as N
    from gameoflife.engine import GolEngine
    with pytest.raises(N.GolError) as ei:
        GolEngine(2, 2, topology="ref-clipped")
    assert ei.value.code == N.GOL_EINVAL
    assert "NextStateCellGathererActor.scala" in ei.value.message


def test_visible_extents_that_strand_cells_are_refused():
    # explicit visible extents leaving a column / row two cells away from
    # anything visible: those cells' gatherers have nobody to ask either
    from gameoflife import _native as N
    assert _create(10, 10, vis=(7, 9)) == N.GOL_EINVAL
    assert _create(10, 10, vis=(9, 7)) == N.GOL_EINVAL
    assert _create(10, 10, vis=(9, 9)) in (N.GOL_OK, N.GOL_ENODEV)


def test_torus_tiny_boards_still_accepted():
    # the torus is the build's own topology (no reference counterpart): its
    # 1- and 2-row boards wrap onto themselves and are tested on the GPU
    from gameoflife import _native as N
    from gameoflife.engine import GolEngine
    for H in (1, 2):
        try:
            GolEngine(32, H, topology="torus").close()
        except N.GolError as e:
            assert e.code == N.GOL_ENODEV


def test_width_beyond_int32_rows_refused():
    """Kernel row pitches are 32-bit word counts: gol_create refuses rows of
    2^31 cells or more before it looks for a device."""
    from gameoflife import _native as N
    from gameoflife.engine import GolEngine
    for W in (1 << 31, 1 << 40):
        try:
            GolEngine(W, 1, topology="torus").close()
            raise AssertionError("accepted")
        except N.GolError as e:
            assert e.code == N.GOL_EINVAL and "2^31" in str(e)
