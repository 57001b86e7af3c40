"""Logging set-up identical in format to the reference (``scripts/train.py:57-61``)."""
from __future__ import annotations

import logging
import sys

LOG_FORMAT = "%(asctime)s - %(name)s - %(levelname)s - %(message)s"


def setup_logging(rank: int = 0, level: str = "INFO", all_ranks: bool = False) -> None:
    """Root ``basicConfig`` at INFO to stdout. Non-zero ranks log WARNING+ unless ``all_ranks``.

    The reference logs from every rank (and shows the Keras progress bar only on rank 0,
    ``scripts/train.py:152``); we keep the rank-0 verbosity and silence duplicate INFO lines.
    """
    lvl = logging.getLevelName(level)
    if rank != 0 and not all_ranks:
        lvl = logging.WARNING
    logging.basicConfig(level=lvl, handlers=[logging.StreamHandler(sys.stdout)], format=LOG_FORMAT, force=True)


def get_logger(name: str) -> logging.Logger:
    return logging.getLogger(name)
