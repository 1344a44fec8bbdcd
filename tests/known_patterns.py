"""Published Life facts (B3/S23 on an unbounded plane) used as known-answer
vectors: they pin the rule independently of the oracle.  Each pattern sits
at the centre of a torus wide enough that nothing it emits wraps around
within the checked generations (gliders move one cell per 4 generations).

* R-pentomino: stabilises at generation 1103 with 116 cells (118 at 1102).
* Diehard: vanishes at generation 130 (2 cells at 129).
* Acorn: stabilises at generation 5206 with 633 cells (635 at 5205).
* Gosper glider gun: 36 cells, period 30, one 5-cell glider per period, so
  36 + 5n cells at generation 30n while no glider has wrapped.
* Pulsar: period 3, populations 48, 56, 72.

Coordinates are (x, y) offsets from the board centre, y growing downwards."""
import numpy as np

R_PENTOMINO = [(1, 0), (2, 0), (0, 1), (1, 1), (1, 2)]
DIEHARD = [(6, 0), (0, 1), (1, 1), (1, 2), (5, 2), (6, 2), (7, 2)]
ACORN = [(1, 0), (3, 1), (0, 2), (1, 2), (4, 2), (5, 2), (6, 2)]

GOSPER_GUN_ROWS = [
    "........................O...........",
    "......................O.O...........",
    "............OO......OO............OO",
    "...........O...O....OO............OO",
    "OO........O.....O...OO..............",
    "OO........O...O.OO....O.O...........",
    "..........O.....O.......O...........",
    "...........O...O....................",
    "............OO......................",
]
PULSAR_ROWS = [
    "..OOO...OOO..",
    ".............",
    "O....O.O....O",
    "O....O.O....O",
    "O....O.O....O",
    "..OOO...OOO..",
    ".............",
    "..OOO...OOO..",
    "O....O.O....O",
    "O....O.O....O",
    "O....O.O....O",
    ".............",
    "..OOO...OOO..",
]


def _cells(rows, cx, cy):
    return [(x - cx, y - cy) for y, r in enumerate(rows) for x, c in enumerate(r) if c == "O"]


GOSPER_GUN = _cells(GOSPER_GUN_ROWS, 18, 4)
PULSAR = _cells(PULSAR_ROWS, 6, 6)

# (name, cells, torus edge, [(generation, population), ...])
CASES = [
    ("r_pentomino", R_PENTOMINO, 1024, [(1102, 118), (1103, 116), (1105, 116)]),
    ("diehard", DIEHARD, 256, [(129, 2), (130, 0), (132, 0)]),
    ("acorn", ACORN, 4096, [(5205, 635), (5206, 633), (5208, 633)]),
    ("gosper_gun", GOSPER_GUN, 512, [(0, 36), (30, 41), (150, 61), (300, 86)]),
    ("pulsar", PULSAR, 64, [(1, 56), (2, 72), (3, 48), (100, 56)]),
]


def board(pack, W, cells):
    c = np.zeros((W, W), dtype=np.uint8)
    for x, y in cells:
        c[W // 2 + y, W // 2 + x] = 1
    return pack(c)


def population(packed):
    return int(np.unpackbits(np.ascontiguousarray(packed).view(np.uint8)).sum())
