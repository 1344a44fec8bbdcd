"""gameoflife -- MI355X-native generation step for almendar/akka-game-of-life.

Mirrors the reference package ``gameoflife`` (src/main/scala/gameoflife/):

* ``board``   -- package.scala / BoardCreator.scala / LoggerActor.scala host
                 logic (neighbourhood, coordinates, NextStep driver, log format);
* ``engine``  -- ``GolEngine``: one libgol shard context (the backend worker
                 that replaces CellActor + NextStateCellGathererActor);
* ``shard``   -- row-block decomposition and the multi-rank driver;
* ``rules``   -- Life-like (birth, survive) masks incl. the reference's rules.

``engine`` (and everything that computes) needs ``lib/libgol.so``; it raises
on import when the library is missing -- there is no CPU fallback.
"""
from .rules import LIFE, REF_EFFECTIVE, REF_LITERAL, Rule, rule_by_name  # noqa: F401

__all__ = ["LIFE", "REF_EFFECTIVE", "REF_LITERAL", "Rule", "rule_by_name", "GolEngine"]


def __getattr__(name):
    if name == "GolEngine":
        from .engine import GolEngine
        return GolEngine
    raise AttributeError(name)
