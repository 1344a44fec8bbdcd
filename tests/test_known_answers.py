"""CPU: the oracle reproduces published Life facts (tests/known_patterns.py)
-- a check of its B3/S23 rule that does not go through the oracle's own
tables.  The GPU kernels are held to the same numbers in
tests/test_gpu_known_answers.py."""
import pytest

from oracle import oracle as O
from known_patterns import CASES, board, population


@pytest.mark.parametrize("name,cells,W,checks", [c for c in CASES if c[0] != "acorn"], ids=lambda v: v if isinstance(v, str) else "")
def test_oracle_reproduces_published_populations(name, cells, W, checks):
    b, done = board(O.pack, W, cells), 0
    for gen, want in checks:
        b, _ = O.run_packed(b, W, gen - done, O.TORUS, O.LIFE)
        done = gen
        assert population(b) == want, (name, gen)
