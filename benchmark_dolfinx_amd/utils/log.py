"""Rank-aware levelled logger.

The reference logs through spdlog with the level taken from unregistered
argv options such as ``SPDLOG_LEVEL=info`` (src/main.cpp:189,229).  The same
argv form is accepted here, as is the env var BENCH_LOG_LEVEL.
"""

from __future__ import annotations

import logging
import os
import sys

_LOGGER = logging.getLogger("bench_dolfinx")


def init_logging(argv=None, rank: int = 0) -> logging.Logger:
    level = os.environ.get("BENCH_LOG_LEVEL", "warning")
    for a in argv or []:
        if a.startswith("SPDLOG_LEVEL=") or a.startswith("--log_level="):
            level = a.split("=", 1)[1]
    lvl = getattr(logging, level.upper(), logging.WARNING)
    _LOGGER.handlers.clear()
    h = logging.StreamHandler(sys.stderr)
    h.setFormatter(logging.Formatter(f"[%(asctime)s] [rank {rank}] [%(levelname)s] %(message)s"))
    _LOGGER.addHandler(h)
    _LOGGER.setLevel(lvl)
    _LOGGER.propagate = False
    return _LOGGER


def get_logger() -> logging.Logger:
    return _LOGGER
