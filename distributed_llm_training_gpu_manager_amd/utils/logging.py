"""Rank-aware logging: every record carries the global rank; non-zero ranks log WARNING+ only
unless DLGM_LOG_ALL_RANKS=1 (keeps 8-rank runs readable)."""
from __future__ import annotations

import logging
import os
import sys


def get_logger(name: str = "dlgm") -> logging.Logger:
    log = logging.getLogger(name)
    if getattr(log, "_dlgm_configured", False):
        return log
    rank = int(os.environ.get("RANK", "0"))
    h = logging.StreamHandler(sys.stderr)
    h.setFormatter(logging.Formatter(f"%(asctime)s [rank{rank}] %(levelname)s %(name)s: %(message)s"))
    log.addHandler(h)
    all_ranks = os.environ.get("DLGM_LOG_ALL_RANKS", "0") == "1"
    log.setLevel(os.environ.get("DLGM_LOG_LEVEL", "INFO") if rank == 0 or all_ranks else "WARNING")
    log.propagate = False
    log._dlgm_configured = True
    return log
