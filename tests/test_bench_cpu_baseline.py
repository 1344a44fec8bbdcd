"""bench.py's cpu_baseline leg: the bit-packed OpenMP port
as the line's value, the scalar per-cell oracle on the 4096^2 torus (one
thread, end state checked against tests/golden/golden.json), and the
reference's derived Akka ceiling -- each with its own kind.  Runs the real
oracle on a short budget (the scalar leg always completes one 4096^2
generation, ~1 s here)."""
import bench


def test_cpu_baseline_has_the_three_figures():
    cb = bench.cpu_baseline(2048, 0.2)
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1
    pp, sc, ak = cb["packed_port"], cb["scalar_4096"], cb["akka_derived_ceiling"]
    assert pp["value"] == cb["value"] and pp["kind"] == "port" and "2048x1024" in pp["sample"]
    assert sc["kind"] == "port" and sc["cores"] == 1 and sc["value"] > 0 and "4096x4096" in sc["sample"]
    assert sc["parity"]["match"] is True and sc["parity"]["epoch"] >= 1
    assert ak["kind"] == "derived" and abs(ak["cell_updates_per_s"] - 49 / 3) < 1e-3
    assert abs(ak["value"] - 49 / 3 / 1e9) < 1e-15 and "application.conf:40" in ak["sample"]
    # the bit-sliced port is far faster than the scalar restatement, which is
    # far faster than the reference's tick-bound ceiling
    assert pp["value"] > sc["value"] > ak["value"]
