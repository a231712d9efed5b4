"""Rank-aware logging (the reference only ``print``s, ref.py:167-255).

``get_logger(name)`` returns a ``cml.*`` logger whose records carry ``[rank r/W]``. By default
only rank 0 emits (SPMD ranks would print the same line W times); ``CML_LOG_ALL_RANKS=1`` lets
every rank log. Level: ``CML_LOG_LEVEL`` (default WARNING) or ``SparkContext.setLogLevel``.
"""
from __future__ import annotations

import logging
import os

_CONFIGURED = False


class _RankFilter(logging.Filter):
    def filter(self, record: logging.LogRecord) -> bool:
        rank = int(os.environ.get("RANK", "0"))
        world = int(os.environ.get("WORLD_SIZE", "1"))
        record.rank_tag = f"[rank {rank}/{world}]"
        return rank == 0 or os.environ.get("CML_LOG_ALL_RANKS", "0") == "1"


def configure() -> None:
    global _CONFIGURED
    if _CONFIGURED:
        return
    _CONFIGURED = True
    root = logging.getLogger("cml")
    if not root.handlers:
        h = logging.StreamHandler()
        h.setFormatter(logging.Formatter("%(asctime)s %(rank_tag)s %(name)s %(levelname)s: %(message)s"))
        h.addFilter(_RankFilter())
        root.addHandler(h)
        root.propagate = False
    root.setLevel(os.environ.get("CML_LOG_LEVEL", "WARNING").upper())


def get_logger(name: str = "cml") -> logging.Logger:
    configure()
    return logging.getLogger(name if name.startswith("cml") else f"cml.{name}")
