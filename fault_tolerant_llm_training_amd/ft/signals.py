"""Preemption signals as flags, never as asynchronous exceptions.

The reference registers ``catch_SIG_exception`` for SIGUSR1/SIGTERM
(reference ``train.py:89-90``), which raises ``Exception("Exception", signum)``
from inside the handler (``utils.py:93-97``). CPython runs that handler at the
next bytecode boundary of the main thread, so the exception can tear an
optimizer step in half or land between ``optimizer.step()`` and
``training_step += 1``, and a second signal during the save
interrupts the save itself (§A.6).

Here the handler is the native ``sigaction`` handler in
``csrc/runtime/signals.cpp`` (lock-free atomic stores only, async-signal-safe);
the trainer polls :meth:`SignalMonitor.pending` at step boundaries, agrees on it
across data-parallel ranks, and then raises :class:`SignalInterrupt` through
the same ``except`` → ``handle_exit`` path the reference uses. Without the
native runtime a Python handler that only sets a flag is used instead.
"""
from __future__ import annotations

import contextlib
import signal
import threading
from typing import Iterable, List, Optional

from .._native import runtime, runtime_available

DEFAULT_SIGNALS = (signal.SIGUSR1, signal.SIGTERM)


class SignalInterrupt(Exception):
    """Raised by the trainer at a step boundary for a pending signal.

    ``args == ("Exception", signum)`` like the reference's handler-raised
    exception (utils.py:97), so code that inspects ``e.args[1]`` still works.
    """

    def __init__(self, signum: int):
        super().__init__("Exception", int(signum))
        self.signum = int(signum)


class SignalMonitor:
    def __init__(self, signums: Iterable[int] = DEFAULT_SIGNALS, native: Optional[bool] = None):
        self.signums: List[int] = [int(s) for s in signums]
        self.native = runtime_available() if native is None else native
        self._py_first = 0
        self._py_count = 0
        self._py_lock = threading.Lock()
        self._installed = False
        self._old = {}

    # -------------------------------------------------------------- install
    def install(self) -> "SignalMonitor":
        if self.native:
            runtime().signals_clear()
            runtime().signals_install(self.signums)
        else:
            for s in self.signums:
                self._old[s] = signal.signal(s, self._py_handler)
        self._installed = True
        return self

    def uninstall(self) -> None:
        if not self._installed:
            return
        if self.native:
            runtime().signals_restore_default(self.signums)
        else:
            for s, h in self._old.items():
                signal.signal(s, h if h is not None else signal.SIG_DFL)
        self._installed = False

    def _py_handler(self, signum, _frame):
        if self._py_first == 0:
            self._py_first = int(signum)
        self._py_count += 1

    # -------------------------------------------------------------- query
    def pending(self) -> int:
        """First signal received since :meth:`clear` (0 if none)."""
        if self.native:
            return int(runtime().signals_pending())
        return self._py_first

    def count(self) -> int:
        if self.native:
            return int(runtime().signals_count())
        return self._py_count

    def clear(self) -> None:
        if self.native:
            runtime().signals_clear()
        else:
            self._py_first = 0

    @contextlib.contextmanager
    def blocked(self):
        """Defer delivery of the monitored signals (e.g. around the final checkpoint publish)."""
        old = signal.pthread_sigmask(signal.SIG_BLOCK, self.signums)
        try:
            yield
        finally:
            signal.pthread_sigmask(signal.SIG_SETMASK, old)
