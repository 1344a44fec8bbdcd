"""Host-side mirror of the reference's frontend around the generation step.

Same names and argument meaning as the reference (src/main/scala/gameoflife/):

* ``generate_neighbour_addresses``  package.scala:17-28
* ``generate_all_coordinates``      BoardCreator.scala:47-53
* ``SimulationParams``              BoardCreator.scala:13-14 (+ application.conf:29-47)
* ``BoardCreator``                  BoardCreator.scala:18-155: StartSimulation,
                                    NextStep, Pause/ResumeSimulation,
                                    SendMeMyNeighbours -- driving a GPU backend
                                    instead of one actor per cell
* ``LoggerActor``                   LoggerActor.scala:11-48: the "At epoch:N"
                                    board dump (positional, see note there)

Only the generation step itself runs on the GPU (``engine.GolEngine``).
"""
from __future__ import annotations

import dataclasses
import re
from typing import Callable, Iterable

import numpy as np

Position = tuple[int, int]
BoardSize = tuple[int, int]


def generate_neighbour_addresses(board_size: BoardSize, position: Position) -> list[Position]:
    """package.scala:17-28: Moore neighbours of (x, y) inside [0,w) x [0,h),
    excluding the cell itself, in the reference's (i outer, j inner) order."""
    (w, h), (x, y) = board_size, position
    moves = (-1, 0, 1)
    return [(x + i, y + j) for i in moves for j in moves
            if 0 <= x + i < w and 0 <= y + j < h and (x + i, y + j) != (x, y)]


def generate_all_coordinates(board_size: BoardSize) -> list[Position]:
    """BoardCreator.scala:47-53: i in 0 to w, j in 0 to h (inclusive ranges),
    so a board of size (w, h) has (w+1) * (h+1) cells."""
    w, h = board_size
    return [(i, j) for i in range(w + 1) for j in range(h + 1)]


def board_cells(board_size: BoardSize) -> tuple[int, int]:
    """(width, height) in cells of the reference board of size (w, h)."""
    return board_size[0] + 1, board_size[1] + 1


@dataclasses.dataclass
class SimulationParams:
    """BoardCreator.scala:13-14, defaults from application.conf:37-47 (ms)."""
    start_delay_ms: int = 1000
    tick_ms: int = 3000
    first_error_after_ms: int = 10000
    error_every_ms: int = 15000
    max_number_of_crashes: int = 100


class LoggerActor:
    """LoggerActor.scala:30-46 output format.

    For a board of size (x, y) the reference prints, per epoch, ``At
    epoch:N``, a dash line of length 2x+1 (:42), y rows (:40) of x entries
    each (:17 slices x messages per row) as ``[a,b,...]`` (:19) and a
    closing dash line followed by an empty line (:44).  It prints once x*y
    CellStateMsgs of the epoch have arrived (:28,35) -- of the (x+1)*(y+1)
    cells the board holds (BoardCreator.scala:47-53) -- filling the rows in
    arrival order (:32-33 prepend).  The arrival order cannot be reproduced;
    the shape can: this logger prints the x*y cells of columns 0..x-1 and
    rows 0..y-1, positionally.  ``full=True`` is this build's extension:
    every row and column of the board (same format, dash line 2w+1 for a
    board w cells wide).  The native frontend (csrc/gol_frontend.cpp) prints
    the same text (``log.full``).
    """

    def __init__(self, board_size: BoardSize, sink: Callable[[str], None] | None = None, full: bool = False):
        self.board_size = board_size
        self.full = full
        self.lines: list[str] = []
        self.sink = sink or self.lines.append

    @staticmethod
    def format_epoch(cells: np.ndarray, epoch: int, size: BoardSize | None = None) -> list[str]:
        """The epoch's text.  size = (x, y): the reference's shape, y rows of
        x entries (cells[:y, :x]); None: all of `cells` (the full-board
        extension)."""
        if size is not None:
            x, y = size
            cells = cells[:y, :x]
        h, w = cells.shape
        rows = ["[" + ",".join(str(int(v)) for v in cells[r]) + "]" for r in range(h)]
        dash = "-" * (w * 2 + 1)
        return [f"At epoch:{epoch}", dash, *rows, dash + "\n"]

    def log_board(self, cells: np.ndarray, epoch: int) -> None:
        for line in self.format_epoch(cells, epoch, None if self.full else self.board_size):
            self.sink(line)


class BoardCreator:
    """Frontend coordinator (BoardCreator.scala:18-155) over GPU backends.

    ``backend`` is any object with ``step(n, hashes)``, ``snapshot()``,
    ``epoch`` -- a ``GolEngine`` (one GPU shard) or a ``ShardGroup``.  The
    reference broadcasts ``CurrentEpochMsg(step)`` to every cell on each
    ``NextStep`` tick (:113-116) and each cell catches up one generation at a
    time (CellActor.scala:41-47,86); here ``next_step`` advances the backend
    to the new global epoch in one call.
    """

    def __init__(self, board_size: BoardSize, params: SimulationParams | None = None,
                 backend=None, logger: LoggerActor | None = None, log_every: int = 0):
        self.board_size = board_size
        self.params = params or SimulationParams()
        self.backend = backend
        self.logger = logger
        self.log_every = log_every
        self.step = 0            # BoardCreator.scala:27
        self.running = False
        self.hashes: list[int] = []

    # BoardCreator.scala:105-108
    def start_simulation(self) -> None:
        if self.backend is None:
            raise RuntimeError("no backend: the reference fails here too "
                               "(Random.nextInt(0) with no backend up, BoardCreator.scala:34-35)")
        self.running = True

    # :109-110
    def pause_simulation(self) -> None:
        self.running = False

    # :111-112
    def resume_simulation(self) -> None:
        self.running = True

    # :113-116 NextStep: step += 1, every cell -> CurrentEpochMsg(step)
    def next_step(self, generations: int = 1) -> list[int]:
        if not self.running:
            return []
        self.step += generations
        hashes = self.backend.step(generations, hashes=True)
        hs = [int(h) for h in hashes]
        self.hashes.extend(hs)
        if self.logger is not None and self.log_every and self.step % self.log_every == 0:
            from . import codec
            cells = codec.unpack(self.backend.snapshot(), self.board_size[0] + 1)
            self.logger.log_board(cells, self.step)
        return hs

    # :117-118 SendMeMyNeighbours(position)
    def send_me_my_neighbours(self, position: Position) -> list[Position]:
        return generate_neighbour_addresses(self.board_size, position)


# ---------------------------------------------------------------- config

_DEFAULTS = {
    "game-of-life.board.size.x": 6,                     # application.conf:32
    "game-of-life.board.size.y": 6,                     # application.conf:33
    "game-of-life.simulation.wait-for-backends": "5s",  # :38
    "game-of-life.simulation.start-delay": "1s",        # :39
    "game-of-life.simulation.tick": "3000ms",           # :40
    "game-of-life.simulation.max-crashes": 100,         # :41
    "game-of-life.errors.delay": "10second",            # :45
    "game-of-life.errors.every": "15seconds",           # :46
    # keys added by this build (SURVEY.md section 5, config/flag system)
    "game-of-life.board.topology": "ref-clipped",
    "game-of-life.simulation.rule": "ref-effective",
    "game-of-life.simulation.seed": 0x5EED,
    "game-of-life.simulation.generations": 100,
    "game-of-life.simulation.gpus": 1,
    "game-of-life.simulation.checkpoint-every": 0,
    "game-of-life.simulation.halo-depth": 1,
}


def parse_duration_ms(v) -> int:
    """Typesafe-config style durations: 3000ms, 5s, 10second, 15seconds."""
    if isinstance(v, (int, float)):
        return int(v)
    m = re.fullmatch(r"\s*(\d+)\s*(ms|millis|milliseconds?|s|seconds?|m|minutes?)?\s*", str(v))
    if not m:
        raise ValueError(f"bad duration {v!r}")
    n, unit = int(m.group(1)), (m.group(2) or "ms")
    if unit.startswith("m") and unit not in ("m", "minute", "minutes"):
        return n
    if unit in ("m", "minute", "minutes"):
        return n * 60000
    return n * 1000


def parse_hocon(text: str) -> dict:
    """Minimal HOCON reader for application.conf-style files: nested blocks,
    ``key = value`` / ``key=value``, // and # comments.  Flattens to dotted keys."""
    out: dict = {}
    stack: list[str] = []
    for raw in text.splitlines():
        line = re.sub(r"(//|#).*$", "", raw).strip()
        if not line:
            continue
        if line.endswith("{"):
            stack.append(line[:-1].strip())
            continue
        if line == "}":
            stack.pop()
            continue
        m = re.fullmatch(r"([\w.\-\"]+)\s*[=:]\s*(.+)", line)
        if not m:
            continue
        key = ".".join(stack + [m.group(1).strip('"')])
        val = m.group(2).strip().strip('"')
        out[key] = int(val) if re.fullmatch(r"-?\d+", val) else val
    return out


def load_config(text: str | None = None, overrides: dict | None = None) -> dict:
    cfg = dict(_DEFAULTS)
    if text:
        cfg.update({k: v for k, v in parse_hocon(text).items() if k.startswith("game-of-life.")})
    if overrides:
        cfg.update(overrides)
    return cfg


def simulation_params(cfg: dict) -> SimulationParams:
    """Run.scala:38-44."""
    return SimulationParams(
        start_delay_ms=parse_duration_ms(cfg["game-of-life.simulation.start-delay"]),
        tick_ms=parse_duration_ms(cfg["game-of-life.simulation.tick"]),
        first_error_after_ms=parse_duration_ms(cfg["game-of-life.errors.delay"]),
        error_every_ms=parse_duration_ms(cfg["game-of-life.errors.every"]),
        max_number_of_crashes=int(cfg["game-of-life.simulation.max-crashes"]),
    )


def crash_schedule(params: SimulationParams, generations: int, seed: int = 0) -> list[tuple[int, int]]:
    """Injected crashes in generations, from the reference's wall-clock
    schedule (BoardCreator.scala:97-102,107-108): NextStep fires at
    start-delay + k * tick and advances to epoch k + 1; crashIfIMay fires at
    errors.delay + i * errors.every and crashes a random child while fewer than
    max-crashes have been crashed.  Crash i therefore lands after epoch
    floor((delay + i * every - start) / tick) + 1.  Each entry is
    (generation, pick): pick is the seeded stand-in for
    Random.nextInt(children.size) (BoardCreator.scala:91-95) -- the victim is
    live shard `pick % live_count`."""
    import random
    rng = random.Random(seed)
    out = []
    for i in range(params.max_number_of_crashes):
        t = params.first_error_after_ms + i * params.error_every_ms
        if t < params.start_delay_ms:
            continue
        g = (t - params.start_delay_ms) // params.tick_ms + 1
        if g > generations:
            break
        out.append((int(g), rng.randrange(1 << 30)))
    return out


def iter_positions(cells: np.ndarray) -> Iterable[tuple[Position, bool]]:
    """(position, state) pairs in generateAllCoordinates order -- the payload
    of the reference's CellStateMsg stream for one epoch."""
    H, W = cells.shape
    for i in range(W):
        for j in range(H):
            yield (i, j), bool(cells[j, i])
