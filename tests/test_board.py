"""CPU tests of the host-side mirror of the reference frontend
(package.scala, BoardCreator.scala, LoggerActor.scala, Run.scala config)."""
import numpy as np
import pytest

from gameoflife import board as B
from gameoflife import rules as R
from oracle import oracle as O


def test_neighbour_addresses_match_reference_semantics():
    # package.scala:17-28 on the default 6x6 board
    assert B.generate_neighbour_addresses((6, 6), (0, 0)) == [(0, 1), (1, 0), (1, 1)]
    assert len(B.generate_neighbour_addresses((6, 6), (3, 3))) == 8
    # column/row w, h are outside [0,w) x [0,h): the corner (6,6) only sees (5,5)
    assert B.generate_neighbour_addresses((6, 6), (6, 6)) == [(5, 5)]
    assert B.generate_neighbour_addresses((6, 6), (6, 0)) == [(5, 0), (5, 1)]
    # i outer, j inner order
    assert B.generate_neighbour_addresses((6, 6), (2, 2))[:3] == [(1, 1), (1, 2), (1, 3)]


def test_neighbourhood_is_the_oracle_clipped_topology():
    """Counting live cells over generate_neighbour_addresses == the oracle's
    REF_CLIPPED count, cell by cell, on random 7x7 boards."""
    rng = np.random.default_rng(5)
    for _ in range(5):
        cells = (rng.random((7, 7)) < 0.5).astype(np.uint8)
        nxt = O.step_cells(cells, O.REF_CLIPPED, O.LIFE)
        for (x, y) in B.generate_all_coordinates((6, 6)):
            n = sum(int(cells[ny, nx]) for nx, ny in B.generate_neighbour_addresses((6, 6), (x, y)))
            want = (n == 3) or (cells[y, x] and n == 2)
            assert bool(nxt[y, x]) == want


def test_all_coordinates_inclusive():
    c = B.generate_all_coordinates((6, 6))
    assert len(c) == 49 and c[0] == (0, 0) and c[1] == (0, 1) and c[-1] == (6, 6)
    assert B.board_cells((6, 6)) == (7, 7)


def test_iter_positions_follows_generate_all_coordinates():
    # the CellStateMsg payload order: x-major, (x, y) with cells[y, x]
    cells = (np.random.default_rng(3).random((7, 7)) < 0.5).astype(np.uint8)
    got = list(B.iter_positions(cells))
    assert [p for p, _ in got] == B.generate_all_coordinates((6, 6))
    assert all(s == bool(cells[y, x]) for (x, y), s in got)


def test_logger_format():
    cells = np.array([[1, 0, 1], [0, 1, 0], [0, 0, 0]], dtype=np.uint8)
    lines = B.LoggerActor.format_epoch(cells, 4)
    assert lines == ["At epoch:4", "-------", "[1,0,1]", "[0,1,0]", "[0,0,0]", "-------\n"]


def test_logger_reference_shape_at_default_board():
    """Board size (6, 6): the reference prints 2x+1 = 13 dashes and y = 6
    rows of x = 6 entries (LoggerActor.scala:17,28,36-44), of the 7 x 7 cells
    the board holds; full=True prints all 7 x 7 (this build's extension)."""
    cells = O.java_random_cells(6, 6, 42)
    out = []
    B.LoggerActor((6, 6), sink=out.append).log_board(cells, 3)
    assert out[0] == "At epoch:3" and out[1] == "-" * 13 and out[-1] == "-" * 13 + "\n"
    rows = out[2:-1]
    assert len(rows) == 6 and all(len(r[1:-1].split(",")) == 6 for r in rows)
    assert rows == ["[" + ",".join(str(int(v)) for v in cells[y, :6]) + "]" for y in range(6)]
    full = []
    B.LoggerActor((6, 6), sink=full.append, full=True).log_board(cells, 3)
    assert full[1] == "-" * 15 and len(full) == 7 + 3 and full[2:-1][:6] != rows
    # non-square size (x, y) = (4, 2): 2 rows of 4
    lines = B.LoggerActor.format_epoch(O.java_random_cells(4, 2, 1), 1, size=(4, 2))
    assert lines[1] == "-" * 9 and len(lines) == 2 + 3 and all(len(r.split(",")) == 4 for r in lines[2:-1])


def test_config_keys_and_durations():
    text = """
    // same shape as the reference's application.conf game-of-life section
    game-of-life {
      board { size { x = 12
                     y = 9 } }
      simulation {
        tick = 250ms
        max-crashes = 3
        seed = 77
      }
      errors { every = 2seconds }
    }
    """
    # the one-line nested block above is not HOCON-canonical; use a clean one too
    text2 = "game-of-life {\n board {\n size {\n x = 12\n y = 9\n }\n }\n simulation {\n" \
            " tick = 250ms\n max-crashes = 3\n seed = 77\n }\n errors {\n every = 2seconds\n }\n}\n"
    cfg = B.load_config(text2)
    assert cfg["game-of-life.board.size.x"] == 12 and cfg["game-of-life.board.size.y"] == 9
    p = B.simulation_params(cfg)
    assert p.tick_ms == 250 and p.max_number_of_crashes == 3 and p.error_every_ms == 2000
    assert p.start_delay_ms == 1000 and p.first_error_after_ms == 10000  # defaults (conf :39,:45)
    assert B.parse_duration_ms("5s") == 5000 and B.parse_duration_ms("1minute") == 60000
    assert B.load_config(text) is not None


def test_rules():
    assert R.rule_by_name("life") == R.LIFE and R.LIFE.notation() == "B3/S23"
    assert R.REF_LITERAL.notation() == "B/S01245678"
    assert R.REF_EFFECTIVE.notation() == "B/S012345678"
    r = R.rule_by_name("B36/S23")
    assert (r.birth, r.survive) == (0x48, 0x0C)
    with pytest.raises(ValueError):
        R.rule_by_name("nope")


class _OracleBackend:
    """Test double standing in for a GPU shard (host-logic test only)."""

    def __init__(self, cells, rule):
        self.W = cells.shape[1]
        self.p = O.pack(cells)
        self.rule = rule
        self.epoch = 0

    def step(self, n, hashes=True):
        self.p, h = O.run_packed(self.p, self.W, n, O.REF_CLIPPED, self.rule)
        self.epoch += n
        return h

    def snapshot(self):
        return self.p


def test_board_creator_drives_backend_and_logs():
    cells = O.java_random_cells(6, 6, 42)
    logger = B.LoggerActor((6, 6))
    bc = B.BoardCreator((6, 6), backend=_OracleBackend(cells, O.REF_EFFECTIVE), logger=logger,
                        log_every=1)
    assert bc.next_step() == []  # not started: ticks do nothing
    bc.start_simulation()
    h1 = bc.next_step()
    h2 = bc.next_step()
    assert bc.step == 2 and h1 == h2  # ref-effective: the board never changes
    bc.pause_simulation()
    assert bc.next_step() == [] and bc.step == 2
    bc.resume_simulation()
    bc.next_step(3)
    assert bc.step == 5
    # logged after ticks reaching epochs 1, 2 and 5 (one multi-generation tick)
    assert logger.lines[0] == "At epoch:1" and len(logger.lines) == 3 * (6 + 3)
    assert logger.lines[18] == "At epoch:5" and logger.lines[1] == "-" * 13
    assert bc.send_me_my_neighbours((0, 0)) == [(0, 1), (1, 0), (1, 1)]


def test_board_creator_without_backend_fails():
    with pytest.raises(RuntimeError):
        B.BoardCreator((6, 6)).start_simulation()
