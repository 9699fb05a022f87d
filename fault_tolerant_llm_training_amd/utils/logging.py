"""Root logger with the reference's exact format.

Parity: reference ``utils.py:10`` (module-global root logger) and
``utils.py:21-29`` (``init_logger``: INFO level, StreamHandler,
``"%(asctime)s - %(name)s - %(levelname)s - %(message)s"``). The log lines are
part of the observable contract, so the format is kept verbatim.
"""
from __future__ import annotations

import logging
import os
import sys

logger = logging.getLogger()

LOG_FORMAT = "%(asctime)s - %(name)s - %(levelname)s - %(message)s"

_initialised = False


def init_logger(rank: int | None = None) -> logging.Logger:
    """Configure the root logger once (idempotent).

    Only rank 0 logs at INFO under data parallelism; other ranks log WARNING and
    above so the Slurm output stays identical to a single-GPU run.
    """
    global _initialised
    if rank is None:
        rank = int(os.environ.get("RANK", os.environ.get("SLURM_PROCID", "0")))
    level = logging.INFO if rank == 0 else logging.WARNING
    logger.setLevel(level)
    if not _initialised:
        ch = logging.StreamHandler(stream=sys.stderr)
        ch.setLevel(logging.INFO)
        ch.setFormatter(logging.Formatter(LOG_FORMAT))
        logger.addHandler(ch)
        _initialised = True
    return logger
