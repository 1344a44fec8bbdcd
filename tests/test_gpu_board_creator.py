"""GPU: the Python frontend mirror (gameoflife.board.BoardCreator +
LoggerActor, BoardCreator.scala:105-116, LoggerActor.scala:30-46) driving a
GolEngine on the reference's default board (size (6, 6): 7 x 7 cells,
ref-clipped) from the golden vectors' java.util.Random boards: every NextStep
tick's hash equals the golden one, and the logger prints the reference's
shape -- 13 dashes, 6 rows of 6 entries -- of the golden board at that
epoch."""
import json
import os

import numpy as np
import pytest

from gameoflife import board as B
from gameoflife.engine import GolEngine
from oracle import oracle as O

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


def _cells(rows):
    return np.array([[int(ch) for ch in r] for r in rows], dtype=np.uint8)


@pytest.mark.parametrize("entry", GOLDEN["ref_default"][:2], ids=lambda e: f"seed{e['java_seed']}")
@pytest.mark.parametrize("rule", ["life", "ref-literal", "ref-effective"])
def test_board_creator_over_gpu_engine(gpu, entry, rule):
    size = (entry["w"], entry["h"])
    res = entry["modes"][rule]
    boards = {b["epoch"]: _cells(b["cells"]) for b in res["boards"]}
    with GolEngine(size[0] + 1, size[1] + 1, topology="ref-clipped", rule=rule) as eng:
        eng.load(O.pack(_cells(entry["initial"])))
        logger = B.LoggerActor(size)
        bc = B.BoardCreator(size, backend=eng, logger=logger, log_every=1)
        bc.start_simulation()
        got = []
        for _ in range(4):  # four NextStep ticks, one generation each
            got += bc.next_step()
        bc.log_every = 100  # logged when the step count is a multiple (BoardCreator.next_step)
        got += bc.next_step(96)  # a tick that has fallen behind: 96 generations in one call
        assert bc.step == 100 and eng.epoch == 100
    assert got == [int(h) for h in res["hashes"]]
    want = []
    for e in (1, 2, 3, 4, 100):
        want += B.LoggerActor.format_epoch(boards[e], e, size=size)
    assert logger.lines == want
    assert logger.lines[1] == "-" * 13 and sum(ln.startswith("[") for ln in logger.lines) == 5 * 6
