"""Exit-policy matrix (reference utils.py:65-90) and the flag-based signal monitor."""
import logging
import os
import signal

import pytest

from fault_tolerant_llm_training_amd._native import runtime_available
from fault_tolerant_llm_training_amd.ft.exit_handler import classify_exception, handle_exit, resubmit_command
from fault_tolerant_llm_training_amd.ft.signals import SignalInterrupt, SignalMonitor

from helpers import sbatch_calls, write_fake_sbatch


class Rec(logging.Handler):
    def __init__(self):
        super().__init__()
        self.msgs = []

    def emit(self, r):
        self.msgs.append(r.getMessage())


@pytest.fixture
def log():
    lg = logging.getLogger("ft-test")
    lg.setLevel(logging.INFO)
    h = Rec()
    lg.addHandler(h)
    yield lg, h.msgs
    lg.removeHandler(h)


def test_classification():
    assert classify_exception(SignalInterrupt(10)) == 10
    assert classify_exception(SignalInterrupt(15)) == 15
    assert classify_exception(Exception("Simulated exception to test signal handler", -1)) == -1
    assert classify_exception(RuntimeError("x")) == -1
    # the reference would read args[1]='No such file' as an unknown signal and not save
    assert classify_exception(OSError(2, "No such file")) == -1
    assert SignalInterrupt(10).args == ("Exception", 10)


@pytest.mark.parametrize("etype,saves,resubmits,first", [
    (10, True, True, "[EXIT HANDLER] Job timed out, saving checkpoint."),
    (-1, True, False, "[EXIT HANDLER] Error during training encountered, saving checkpoint."),
    (15, False, False, "[EXIT HANDLER] Job cancelled, terminating."),
    (7, False, False, "[EXIT HANDLER] Unknown exit signal 7, terminating."),
])
def test_policy_matrix(tmp_path, monkeypatch, log, etype, saves, resubmits, first):
    lg, msgs = log
    d = str(tmp_path)
    write_fake_sbatch(d)
    monkeypatch.setenv("PATH", d + os.pathsep + os.environ["PATH"])
    monkeypatch.setenv("WORKDIR", "/work/dir")
    saved = []
    handle_exit(lambda: saved.append(1), 427, etype, lg, job_id="444664")
    assert msgs[0] == first
    assert bool(saved) == saves
    if saves:
        assert "[EXIT HANDLER] Checkpoint saved at step 427" in msgs
    calls = sbatch_calls(d)
    if resubmits:
        assert calls == [["/work/dir/train.sh", "444664"]]
        assert msgs[-1] == "[EXIT HANDLER] sbatch requeued, new job will load the last checkpoint"
    else:
        assert calls == []


def test_failed_requeue_is_logged(tmp_path, monkeypatch, log):
    lg, msgs = log
    bad = tmp_path / "sbatch"
    bad.write_text("#!/bin/bash\nexit 1\n")
    bad.chmod(0o755)
    monkeypatch.setenv("PATH", str(tmp_path) + os.pathsep + os.environ["PATH"])
    handle_exit(lambda: None, 3, 10, lg, job_id="99")
    assert msgs[-1] == "[EXIT HANDLER] Failed to requeue job 99."


def test_non_main_rank_never_resubmits(tmp_path, monkeypatch, log):
    lg, _ = log
    d = str(tmp_path)
    write_fake_sbatch(d)
    monkeypatch.setenv("PATH", d + os.pathsep + os.environ["PATH"])
    handle_exit(lambda: None, 3, 10, lg, job_id="5", is_main=False)
    assert sbatch_calls(d) == []


def test_resubmit_command_shape(monkeypatch):
    monkeypatch.delenv("FT_SBATCH", raising=False)
    assert resubmit_command("/w/train.sh", "12") == ["sbatch", "/w/train.sh", "12"]


@pytest.mark.parametrize("native", [True, False])
def test_signal_monitor_sets_flag_only(native):
    if native and not runtime_available():
        pytest.skip("native runtime not built")
    mon = SignalMonitor(native=native).install()
    try:
        assert mon.pending() == 0
        os.kill(os.getpid(), signal.SIGUSR1)
        os.kill(os.getpid(), signal.SIGTERM)  # would kill the process without the handler
        for _ in range(1000):
            if mon.pending():
                break
        assert mon.pending() == int(signal.SIGUSR1)  # first signal wins
        assert mon.count() >= 2
        mon.clear()
        assert mon.pending() == 0
        with mon.blocked():  # a late signal during the final save only sets the flag
            os.kill(os.getpid(), signal.SIGTERM)
        for _ in range(1000):
            if mon.pending():
                break
        assert mon.pending() == int(signal.SIGTERM)
    finally:
        mon.uninstall()
