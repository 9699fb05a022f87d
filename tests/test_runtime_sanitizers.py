"""Race detection / memory sanitizers for the native runtime.

The host C++ runtime (async-signal-safe flags, the multi-threaded checkpoint zip writer,
the sharded piece writer, the parallel O_DIRECT reader) is built into a self-test binary
under ASan+UBSan and under ThreadSanitizer (host code only; `_build.build_selftest`) and
run on the CPU. Any sanitizer report or self-check failure fails the test.
"""
import os
import subprocess

import pytest

from fault_tolerant_llm_training_amd import _build

REPORTS = ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer", "ERROR: LeakSanitizer")


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_runtime_selftest_sanitized(kind, tmp_path):
    exe = _build.build_selftest(kind, tmp_path / kind)
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    env["TSAN_OPTIONS"] = "halt_on_error=1:second_deadlock_stack=1"
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "runtime selftest ok" in r.stdout
    for rep in REPORTS:
        assert rep not in out, out[-4000:]
