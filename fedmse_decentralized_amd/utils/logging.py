"""Logging with the reference's format (`src/main.py:32-34`)."""
from __future__ import annotations

import logging
import sys

FORMAT = "%(asctime)s - %(levelname)s - %(message)s"
_configured = False


def setup_logging(level: str = "INFO", rank: int = 0, all_ranks: bool = False) -> logging.Logger:
    global _configured
    log = logging.getLogger("fedmx")
    if not _configured:
        h = logging.StreamHandler(sys.stderr)
        h.setFormatter(logging.Formatter(FORMAT))
        log.addHandler(h)
        log.propagate = False
        _configured = True
    lvl = getattr(logging, str(level).upper(), logging.INFO)
    if rank != 0 and not all_ranks:
        lvl = max(lvl, logging.WARNING)
    log.setLevel(lvl)
    return log
