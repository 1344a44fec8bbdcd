"""GPU: the step kernels reproduce published Life facts
(tests/known_patterns.py) at the pass depths the planner uses and at one
generation per pass -- including acorn's 5206 generations on a 4096^2 torus,
too long for the CPU suite."""
import pytest

from oracle import oracle as O
from known_patterns import CASES, board, population

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("gpp", [0, 1, 7, 10, 12])
@pytest.mark.parametrize("name,cells,W,checks", CASES, ids=lambda v: v if isinstance(v, str) else "")
def test_kernels_reproduce_published_populations(gpu, name, cells, W, checks, gpp):
    from gameoflife.engine import GolEngine
    if gpp == 1 and name == "acorn":
        pytest.skip("5206 single-generation passes: covered at the fused depths")
    with GolEngine(W, W) as e:
        e.set_tuning(gens_per_pass=gpp)
        e.load(board(O.pack, W, cells))
        done = 0
        for gen, want in checks:
            e.step(gen - done)
            done = gen
            assert population(e.snapshot()) == want, (name, gen, gpp)
