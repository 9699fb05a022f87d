"""Exit policy: what to do when training is interrupted.

Same policy matrix and log strings as the reference's ``handle_exit``
(reference ``utils.py:65-90``):

=====================  ======  =====  =========  =======================================
trigger                type    save   resubmit   log
=====================  ======  =====  =========  =======================================
Slurm ``USR1@120``     10      yes    yes        timed out → saved → requeued / failed
Python exception       -1      yes    no         error → saved
``scancel`` SIGTERM    15      no     no         cancelled
anything else          other   no     no         unknown exit signal
=====================  ======  =====  =========  =======================================

Differences by design: the exception *type* decides the code (a
:class:`~.signals.SignalInterrupt` carries its signal number, every other
exception is -1), so an ``OSError(errno, msg)`` now saves a checkpoint instead
of being misread as "unknown signal" (SURVEY.md §A.5); the checkpoint is
written atomically by the checkpoint engine; resubmission uses ``subprocess``
with an argument vector instead of a shell string.
"""
from __future__ import annotations

import os
import signal
import subprocess
import sys
from typing import Callable, Optional

from .signals import SignalInterrupt

SIGUSR1 = int(signal.SIGUSR1)   # 10 on Linux
SIGTERM = int(signal.SIGTERM)   # 15
ERROR = -1


def classify_exception(e: BaseException) -> int:
    """Exit type for an exception caught by the trainer (reference train.py:121-126)."""
    if isinstance(e, SignalInterrupt):
        return e.signum
    return ERROR


def resubmit_command(script: str, job_id: Optional[str]):
    """``sbatch <script> <JOBID>`` (reference utils.py:84 → train.sh:24-27)."""
    cmd = [os.environ.get("FT_SBATCH", "sbatch"), script]
    if job_id:
        cmd.append(str(job_id))
    return cmd


def resubmit(script: str, job_id: Optional[str], logger) -> bool:
    try:
        r = subprocess.run(resubmit_command(script, job_id), capture_output=True, text=True, timeout=120)
    except (OSError, subprocess.SubprocessError) as e:
        logger.error(f"[EXIT HANDLER] sbatch could not be run: {e!r}")
        return False
    if r.stdout:
        sys.stdout.write(r.stdout)
        sys.stdout.flush()
    if r.stderr:
        sys.stderr.write(r.stderr)
        sys.stderr.flush()
    return r.returncode == 0


def handle_exit(save_checkpoint: Callable[[], object], training_step: int, exit_type: int, logger,
                job_id: Optional[str] = None, sbatch_script: str = "", is_main: bool = True,
                rank: int = 0) -> None:
    """Apply the exit policy.

    ``save_checkpoint()`` writes the checkpoint durably (blocking); it is called on
    every rank (the engine decides which ranks write). Only the main rank resubmits.
    The main rank logs the reference's lines; every other rank (which logs at WARNING
    only) reports the same lines once, prefixed with its rank, so a job log shows
    that all ranks stopped and saved at the same step.
    """
    say = logger.info if is_main else (lambda m: logger.warning(f"[rank {rank}] {m}"))
    if exit_type == SIGTERM:
        say("[EXIT HANDLER] Job cancelled, terminating.")
        return
    if exit_type == SIGUSR1:
        say("[EXIT HANDLER] Job timed out, saving checkpoint.")
    elif exit_type == ERROR:
        say("[EXIT HANDLER] Error during training encountered, saving checkpoint.")
    else:
        say(f"[EXIT HANDLER] Unknown exit signal {exit_type}, terminating.")
        return
    if save_checkpoint() is False:
        logger.error(f"[EXIT HANDLER] Checkpoint could not be saved at step {training_step}")
        return
    say(f"[EXIT HANDLER] Checkpoint saved at step {training_step}")
    if exit_type == SIGUSR1 and is_main:
        script = sbatch_script or os.path.join(os.getenv("WORKDIR", ""), "train.sh")
        if not resubmit(script, job_id, logger):
            logger.info(f"[EXIT HANDLER] Failed to requeue job {job_id}.")
        else:
            logger.info("[EXIT HANDLER] sbatch requeued, new job will load the last checkpoint")
