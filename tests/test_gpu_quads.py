"""GPU: the opt-in quad layout (GOL_LAYOUT=quads; DESIGN.md section 3 and
section 4 "Quad layout") end to end, in a child process so that libgol and
the oracle read the switch before they are loaded (tests/quads_child.py):
seed, conversions, get_cell, every pass depth hashed and unhashed, quad strip
edges, band heights, generic rules, the 4096^2 x 1000 board and a 2-rank
loopback ring, all bit-exact against the oracle."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_quad_layout_end_to_end(gpu):
    env = dict(os.environ, GOL_LAYOUT="quads")
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "quads_child.py")], env=env,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "QUADS OK" in r.stdout, (r.stdout[-3000:], r.stderr[-3000:])
