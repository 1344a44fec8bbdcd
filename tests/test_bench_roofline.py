"""bench.py's roofline fields (CPU: pure functions over a synthetic PMC
table).  The dominant multi-generation kernel is reported against the VALU
issue ceiling at the guide's 2.4 GHz max clock (frac <= 1 for any rate the
model allows); the clock the launches held prices a separate issue-efficiency
diagnostic; the physical HBM fraction and the 2-bit/cell/generation
'effective' figure sit beside it; single-generation passes stay HBM-bound."""
import bench


def _table(monkeypatch, entries):
    monkeypatch.setattr(bench, "pmc_launch", lambda: entries)


def test_valu_roofline_with_pmc(monkeypatch):
    ent = lambda g, ms, clk: {"launch_ms": ms, "hbm_bytes": 18e9, "clock_ghz": clk, "valu_per_word_gen": 12.0,
                              "generations_per_launch": g}
    _table(monkeypatch, {"262144x262144/N1/G6/h0": ent(6, 4.0, 2.0), "262144x262144/N1/G8/h0": ent(8, 5.0, 1.9)})
    cells = 262144 * 262144
    r = bench.roofline(kms=13.0, launches=3, gens_covered=20, cells=cells, plan=[6, 6, 8],
                       shape="262144x262144", mode="N1")
    assert r["bound"] == "valu" and r["unit"] == "GCUPS" and r["peak_clock_ghz"] == 2.4
    clock = (2.0 * 4 + 2.0 * 4 + 1.9 * 5) / 13
    assert abs(r["held_clock"]["clock_pmc_ghz"] - round(clock, 3)) < 1e-3
    peak = 1024 * 2.4 * 2048 / 26.8  # the guide's max clock, whatever the launches held (pair-row mix)
    achieved = cells * 20 / 3 / (13.0 / 3 / 1e3) / 1e9
    assert abs(r["peak"] - peak) < 1.0 and abs(r["achieved"] - achieved) < 1.0
    assert abs(r["frac"] - achieved / peak) < 1e-3 and r["frac"] < 1
    assert "issue_efficiency" not in r["held_clock"]  # no probe clock given
    assert r["traffic"] == 18e9
    assert r["hbm"]["frac"] < 1 and r["hbm_effective"]["frac"] > 1


def test_missing_pmc_entry(monkeypatch):
    _table(monkeypatch, {})
    r = bench.roofline(kms=10.0, launches=2, gens_covered=16, cells=1 << 30, plan=[8, 8],
                       shape="65536x16384", mode="ring")
    assert r["traffic"] is None and r["held_clock"]["clock_pmc_ghz"] is None and "hbm" not in r
    peak, _ = bench.valu_peak_gcups(bench.VALU_MIX, bench.CLOCK_MAX_GHZ)
    assert abs(r["peak"] - round(peak, 1)) < 0.2


def test_single_generation_passes_are_hbm_bound(monkeypatch):
    _table(monkeypatch, {"65536x65536/N1/G1/h0": {"launch_ms": 0.2, "hbm_bytes": 1.1e9, "clock_ghz": 2.1,
                                                  "valu_per_word_gen": 20.0, "generations_per_launch": 1}})
    r = bench.roofline(kms=20.4, launches=102, gens_covered=102, cells=65536 * 65536, plan=[1] * 102,
                       shape="65536x65536", mode="N1")
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and 0.5 < r["frac"] < 1
    assert r["traffic"] == 1100000000 and r["measured_hbm_frac"] < 1


def test_hashed_mix_adds_the_multiply_add():
    p0, c0 = bench.valu_peak_gcups(bench.VALU_MIX, 2.4)
    p1, c1 = bench.valu_peak_gcups(bench.VALU_MIX_HASH, 2.4)
    assert abs(c1 - c0 - 4.6) < 1e-9 and p1 < p0


def test_pair_row_mix():
    """The pair-layout mix is the row-pair-shared circuit's (8 full-rate logic
    ops per word-generation, 26.8 cycles)."""
    _, c = bench.valu_peak_gcups(bench.VALU_MIX, 2.4)
    assert abs(c - 26.8) < 1e-9
    assert sum(n for k, (n, _) in bench.VALU_MIX.items() if k not in ("v_alignbit_b32", "v_mov_b32_dpp")) == 8


def test_compact_plan_keeps_json_short():
    assert bench.compact_plan([1] * 256) == "256 x 1"
    assert bench.compact_plan([12] * 7 + [9, 9]) == "7 x 12 + 2 x 9"


def test_probe_clock_prices_only_the_issue_efficiency(monkeypatch):
    """The clock measured inside the timed launches (gol_profile_clock) prices
    held_clock.issue_efficiency; frac stays priced at 2.4 GHz."""
    ent = {"launch_ms": 4.0, "hbm_bytes": 18e9, "clock_ghz": 2.2, "valu_per_word_gen": 12.0,
           "generations_per_launch": 12}
    _table(monkeypatch, {"262144x262144/N1/G12/h0": ent})
    r = bench.roofline(kms=12.0, launches=2, gens_covered=24, cells=262144 * 262144, plan=[12, 12],
                       shape="262144x262144", mode="N1", clock=1.9)
    hc = r["held_clock"]
    assert hc["ghz"] == 1.9 and "probe" in hc["source"] and hc["clock_pmc_ghz"] == 2.2
    peak_held, _ = bench.valu_peak_gcups(bench.VALU_MIX, 1.9)
    peak_max, _ = bench.valu_peak_gcups(bench.VALU_MIX, 2.4)
    assert abs(hc["peak_at_held_clock"] - round(peak_held, 1)) < 0.2
    assert abs(r["peak"] - round(peak_max, 1)) < 0.2
    assert abs(hc["issue_efficiency"] * peak_held - r["frac"] * peak_max) < 5
    assert r["frac"] < hc["issue_efficiency"] and r["traffic"] == 18e9


def test_guide_issue_fraction_and_issue_rate(monkeypatch):
    """frac_guide_issue prices the launches at the guide's 2 cycles per wave64
    VALU instruction (10 instructions per word-generation: 20 cycles); the
    issue rate is wave-VALU per cycle per SIMD at the held clock (<= 0.5)."""
    ent = {"launch_ms": 5.4, "hbm_bytes": 17.6e9, "clock_ghz": 2.0, "valu_per_word_gen": 10.2,
           "generations_per_launch": 10}
    _table(monkeypatch, {"262144x262144/N1/G10/h0": ent})
    cells = 262144 * 262144
    r = bench.roofline(kms=10.84, launches=2, gens_covered=20, cells=cells, plan=[10, 10],
                       shape="262144x262144", mode="N1", clock=2.01)
    guide = 1024 * 2.4e9 / 20 * 2048 / 1e9
    assert abs(r["peak_guide_issue"] - guide) < 0.2
    assert abs(r["frac_guide_issue"] - r["achieved"] / guide) < 1e-3 and r["frac_guide_issue"] < r["frac"]
    ir = r["issue_rate"]
    want = r["achieved"] * 1e9 / 2048 * 10.2 / (1024 * 2.01e9)
    assert abs(ir["wave_valu_per_cycle_per_simd"] - want) < 1e-3 and ir["guide_max"] == 0.5
    assert ir["clock_ghz"] == 2.01 and ir["valu_per_word_generation"] == 10.2
    assert "mix-priced" in r["frac_kind"]


def test_issue_rate_uses_the_pmc_clock_without_a_probe(monkeypatch):
    ent = {"launch_ms": 5.4, "hbm_bytes": 17.6e9, "clock_ghz": 2.0, "valu_per_word_gen": 10.0,
           "generations_per_launch": 10}
    _table(monkeypatch, {"262144x262144/N1/G10/h0": ent})
    r = bench.roofline(kms=10.84, launches=2, gens_covered=20, cells=262144 * 262144, plan=[10, 10],
                       shape="262144x262144", mode="N1")
    assert r["issue_rate"]["clock_ghz"] == 2.0 and "PMC clock" in r["issue_rate"]["source"]
    _table(monkeypatch, {})
    r = bench.roofline(kms=10.84, launches=2, gens_covered=20, cells=262144 * 262144, plan=[10, 10],
                       shape="262144x262144", mode="N1")
    assert "issue_rate" not in r  # no clock at all: no rate


def test_copy_peak_and_single_generation_fraction(monkeypatch):
    monkeypatch.setattr(bench, "copy_peak", lambda: {"gbs": 6000.0, "variant": "x", "source": "profiles/copy_peak.json"})
    _table(monkeypatch, {})
    r = bench.roofline(kms=20.4, launches=102, gens_covered=102, cells=65536 * 65536, plan=[1] * 102,
                       shape="65536x65536", mode="N1")
    assert r["copy_peak"]["gbs"] == 6000.0
    assert abs(r["frac_of_copy_peak"] - r["achieved"] / 6000.0) < 1e-3
    r = bench.roofline(kms=10.84, launches=2, gens_covered=20, cells=262144 * 262144, plan=[10, 10],
                       shape="262144x262144", mode="N1")
    assert r["copy_peak"]["source"].startswith("profiles/") and "frac_of_copy_peak" not in r


def test_committed_copy_peak_file():
    """profiles/copy_peak.json, when present, carries the measured rate and
    where it came from."""
    cp = bench.copy_peak()
    if cp is None:
        return
    assert 3000 < cp["gbs"] < bench.HBM_PEAK_GBS and cp["source"].startswith("profiles/copy_peak.json")
