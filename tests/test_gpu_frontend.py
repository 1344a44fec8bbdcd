"""GPU: the native C++ frontend (bin/gol_frontend, a mirror of RunFrontend /
BoardCreator / LoggerActor linked against the C ABI only) reproduces the
golden vectors of the reference's default board (BASELINE.json config 1
geometry), single-shard and as an in-process shard group."""
import json
import os
import subprocess

import numpy as np
import pytest

from gameoflife.board import LoggerActor
from oracle import oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "akka-game-of-life_amd", "bin", "gol_frontend")
GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


def run(args, tmp_path):
    log = tmp_path / "info.log"
    p = subprocess.run([EXE, "--quiet", f"log.file={log}", *args], capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stderr
    hashes = [int(ln.split()[2], 16) for ln in p.stdout.splitlines() if ln.startswith("hash ")]
    return hashes, log.read_text() if log.exists() else ""


@pytest.mark.parametrize("shards", [1, 3])
def test_frontend_reference_board_golden(gpu, tmp_path, shards):
    for entry in GOLDEN["ref_default"][:2]:
        for name, res in entry["modes"].items():
            hashes, text = run([f"simulation.seed={entry['java_seed']}", f"simulation.rule={name}",
                                "simulation.generations=100", "log.every=100",
                                f"simulation.shards={shards}"], tmp_path)
            assert hashes == res["hashes"], (entry["java_seed"], name, shards)
            final = np.array([[int(ch) for ch in row] for row in res["boards"][-1]["cells"]],
                             dtype=np.uint8)
            # the reference's shape at size (6, 6): 13 dashes, 6 rows of 6 entries
            want = "\n".join(LoggerActor.format_epoch(final, 100, size=(6, 6))) + "\n"
            assert text.endswith(want) and want.split("\n")[1] == "-" * 13
            assert want.count("[") == 6 and all(r.count(",") == 5 for r in want.split("\n") if r.startswith("["))
            (tmp_path / "info.log").unlink()


def test_frontend_torus_matches_oracle(gpu, tmp_path):
    hashes, _ = run(["board.topology=torus", "board.size.x=1024", "board.size.y=300", "simulation.rule=life",
                     "simulation.seed=7", "simulation.generations=20", "log.every=0"], tmp_path)
    _, want = O.run_packed(O.seed_packed(1024, 300, 7), 1024, 20, O.TORUS, O.LIFE)
    assert hashes == [int(x) for x in want]


def test_frontend_reads_application_conf(gpu, tmp_path):
    conf = tmp_path / "application.conf"
    conf.write_text("game-of-life {\n  board {\n    size {\n      x = 10\n      y = 8\n    }\n  }\n"
                    "  simulation {\n    tick = 1ms\n    rule = \"B3/S23\"\n    seed = 5\n"
                    "    generations = 7\n  }\n}\n")
    p = subprocess.run([EXE, "--config", str(conf), "log.file=-", "log.every=7"], capture_output=True,
                       text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    assert p.stdout.count("Epoch: ") == 7 and "At epoch:7" in p.stdout
    cells = O.java_random_cells(10, 8, 5)
    final, want = O.run_packed(O.pack(cells), 11, 7, O.REF_CLIPPED, O.LIFE)
    got = [int(ln.split()[2], 16) for ln in p.stdout.splitlines() if ln.startswith("hash ")]
    assert got == [int(x) for x in want]
    assert "\n".join(LoggerActor.format_epoch(O.unpack(final, 11), 7, size=(10, 8))) in p.stdout


def test_frontend_full_board_dump(gpu, tmp_path):
    """log.full=true (this build's extension): every row and column of the
    (x+1) x (y+1) board, 2(x+1)+1 dashes."""
    entry = GOLDEN["ref_default"][0]
    hashes, text = run([f"simulation.seed={entry['java_seed']}", "simulation.rule=life",
                        "simulation.generations=100", "log.every=100", "log.full=true"], tmp_path)
    res = entry["modes"]["life"]
    assert hashes == res["hashes"]
    final = np.array([[int(ch) for ch in row] for row in res["boards"][-1]["cells"]], dtype=np.uint8)
    want = "\n".join(LoggerActor.format_epoch(final, 100)) + "\n"
    assert text.endswith(want) and want.split("\n")[1] == "-" * 15
