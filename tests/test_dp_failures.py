"""Data-parallel failure semantics on the CPU (gloo), world sizes 2 and 4, both gradient modes.

The reference is single-process: any Python exception — including the non-finite
gradient-norm RuntimeError of ``clip_grad_norm_`` — is caught and saved
(reference train.py:121-129, utils.py:61,72-81). Under data parallelism the
same must hold for every rank at the SAME step, whichever rank failed:

* non-finite gradients (``--learning-rate 1e30``) → every rank logs
  "Checkpoint saved at step N" with one N, and the file equals (bit for bit)
  the checkpoint an injected fault at step N writes;
* an ``OSError`` on ONE rank — while fetching its batch, half-way through
  backward (after some gradient buckets went out), or just before the
  optimizer step — → one checkpoint, equal to the fault-at-the-same-step one;
* one rank SIGKILLed (or hung) → the survivors exit within the peer timeout
  instead of blocking for the collective timeout; with replicated state one
  survivor still writes the checkpoint.
"""
import os
import re
import signal
import socket
import subprocess
import sys
import time

import pytest
import torch

from helpers import ROOT, TINY, env_for, kill_group, write_fake_sbatch

pytestmark = pytest.mark.slow

TRAIN = os.path.join(ROOT, "train.py")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(d, job, args, world, extra=None, tag="run"):
    """One process per rank, like ``srun`` (no torchrun agent that would kill the survivors)."""
    port = _port()
    procs = []
    for r in range(world):
        env = env_for(d, job, {"OMP_NUM_THREADS": "1", "RANK": str(r), "WORLD_SIZE": str(world),
                               "LOCAL_RANK": str(r), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        if extra:
            env.update(extra)
        log = open(os.path.join(d, f"{tag}_{job}_r{r}.log"), "w")
        procs.append(subprocess.Popen([sys.executable, TRAIN] + list(args), cwd=d, env=env, stdout=log,
                                      stderr=subprocess.STDOUT, start_new_session=True))
    return procs


def _wait_all(procs, timeout=300):
    t0 = time.time()
    rcs = []
    try:
        for p in procs:
            rcs.append(p.wait(timeout=max(1, timeout - (time.time() - t0))))
    finally:
        for p in procs:
            kill_group(p)
    return rcs, time.time() - t0


def _logs(d, job, world, tag="run"):
    return [open(os.path.join(d, f"{tag}_{job}_r{r}.log")).read() for r in range(world)]


def _base(d, mode, steps=12):
    return TINY + ["--synthetic-data", "--vocab-size", "256", "--training-steps", str(steps),
                   "--lr-warmup-steps", "3", "--dp-mode", mode, "--dp-bucket-mb", "0.05",
                   "--checkpoint-path", os.path.join(d, "ck"), "--logging-frequency", "1"]


def _load(d, job):
    return torch.load(os.path.join(d, "ck", f"checkpoint_{job}.ckpt"), map_location="cpu", weights_only=True)


def _assert_same_state(a, b):
    assert a["training_step"] == b["training_step"]
    for k in a["model"]:
        assert torch.equal(a["model"][k], b["model"][k]), k
    for i in a["optimizer"]["state"]:
        for key in ("exp_avg", "exp_avg_sq", "step"):
            assert torch.equal(a["optimizer"]["state"][i][key], b["optimizer"]["state"][i][key]), (i, key)
    assert a["lr_scheduler"] == b["lr_scheduler"]
    assert [s["next_step"] for s in a["data_loader"]] == [s["next_step"] for s in b["data_loader"]]


def _saved_steps(logs):
    return [int(m.group(1)) for m in (re.search(r"Checkpoint saved at step (\d+)", o) for o in logs) if m]


def _reference_at(d, mode, world, step, args_extra=()):
    """Checkpoint written by the injected fault (all ranks, reference train.py:111-113) at ``step``."""
    job = f"ref{step}{mode}{world}"
    procs = _launch(d, job, _base(d, mode) + list(args_extra) + ["--raise-error", "--error-step", str(step)], world)
    rcs, _ = _wait_all(procs)
    logs = _logs(d, job, world)
    assert rcs == [0] * world and _saved_steps(logs) == [step] * world, logs
    return _load(d, job)


CASES = [(2, "zero1"), (2, "allreduce"), (4, "zero1"), (4, "allreduce")]


@pytest.mark.parametrize("world,mode", CASES)
def test_nonfinite_gradients_save_same_step_on_every_rank(tmp_path, world, mode):
    d = str(tmp_path)
    write_fake_sbatch(d)
    lr = ["--learning-rate", "1e30"]
    procs = _launch(d, "900", _base(d, mode) + lr, world)
    rcs, _ = _wait_all(procs)
    logs = _logs(d, "900", world)
    assert rcs == [0] * world, logs
    steps = _saved_steps(logs)
    assert len(steps) == world and len(set(steps)) == 1, logs
    assert all("Error during training encountered" in o for o in logs), logs
    assert any("is non-finite at optimizer step" in o for o in logs), logs
    n = steps[0]
    assert 0 < n < 12
    _assert_same_state(_load(d, "900"), _reference_at(d, mode, world, n, lr))


@pytest.mark.parametrize("world,mode", CASES)
def test_oserror_inside_backward_on_one_rank(tmp_path, world, mode):
    """Rank 1 fails after its first bucket collective went out: it finishes its share of the
    step with NaN gradients, every rank's guard skips the update, and all save step 5."""
    d = str(tmp_path)
    write_fake_sbatch(d)
    procs = _launch(d, "910", _base(d, mode), world, {"FT_INJECT_FAULT": "1:5:backward"})
    rcs, _ = _wait_all(procs)
    logs = _logs(d, "910", world)
    assert rcs == [0] * world, logs
    assert _saved_steps(logs) == [5] * world, logs
    assert "injected I/O error inside backward" in logs[1]
    _assert_same_state(_load(d, "910"), _reference_at(d, mode, world, 5))


@pytest.mark.parametrize("phase,saved", [("data", 5), ("forward", 5), ("optimizer", 6), ("post", 6)])
def test_oserror_on_one_rank_other_phases(tmp_path, phase, saved):
    d = str(tmp_path)
    write_fake_sbatch(d)
    procs = _launch(d, "920", _base(d, "zero1"), 2, {"FT_INJECT_FAULT": f"1:5:{phase}"})
    rcs, _ = _wait_all(procs)
    logs = _logs(d, "920", 2)
    assert rcs == [0, 0], logs
    # before the step's update: saved at 5; after it (the step completed validly): at 6
    assert _saved_steps(logs) == [saved, saved], logs
    _assert_same_state(_load(d, "920"), _reference_at(d, "zero1", 2, saved))


@pytest.mark.parametrize("world,mode", [(2, "allreduce"), (2, "zero1"), (4, "allreduce")])
def test_sigkilled_rank_survivors_exit_within_bound(tmp_path, world, mode):
    d = str(tmp_path)
    write_fake_sbatch(d)
    args = _base(d, mode, steps=10000) + ["--peer-timeout", "20"]
    procs = _launch(d, "930", args, world, {"FT_INJECT_FAULT": "1:6:kill"})
    try:
        assert procs[1].wait(timeout=180) == -signal.SIGKILL
        t_kill = time.time()
        rcs = [p.wait(timeout=60) for i, p in enumerate(procs) if i != 1]
        waited = time.time() - t_kill
    finally:
        for p in procs:
            kill_group(p)
    logs = _logs(d, "930", world)
    assert rcs == [1] * (world - 1), logs
    assert waited < 30, waited
    survivors = [o for i, o in enumerate(logs) if i != 1]
    assert all("Lost a peer rank" in o for o in survivors), survivors
    saved = _saved_steps(survivors)
    if mode == "allreduce":  # replicated state: exactly one survivor writes it
        assert len(saved) == 1 and saved[0] == 6, survivors
        c = _load(d, "930")
        assert c["training_step"] == 6
        _assert_same_state(c, _reference_at(d, mode, world, 6))
    else:  # ZeRO-1 shards died with the rank: nothing complete to write
        assert saved == [], survivors
        assert not os.path.exists(os.path.join(d, "ck", "checkpoint_930.ckpt"))


def test_hung_rank_detected_after_peer_timeout(tmp_path):
    d = str(tmp_path)
    write_fake_sbatch(d)
    args = _base(d, "allreduce", steps=10000) + ["--peer-timeout", "6"]
    procs = _launch(d, "940", args, 2, {"FT_INJECT_FAULT": "1:4:hang"})
    try:
        t0 = time.time()
        rc0 = procs[0].wait(timeout=120)
        waited = time.time() - t0
    finally:
        for p in procs:
            kill_group(p)
    logs = _logs(d, "940", 2)
    assert rc0 == 1, logs[0]
    assert "Lost a peer rank" in logs[0]
    assert waited < 60, waited


@pytest.mark.parametrize("phase,saved", [("forward", 3), ("post", 4)])
def test_fault_just_before_periodic_save_boundary(tmp_path, phase, saved):
    """The periodic save is collective; it is taken only after the boundary vote passed on
    every rank. Rank 1 fails in step 3 (the save is due at boundary 4): every rank stops at
    that vote and takes the error path's save (step 3 when the step was poisoned, 4 when it
    completed validly) — no rank is left inside the periodic save's collectives."""
    d = str(tmp_path)
    write_fake_sbatch(d)
    args = _base(d, "zero1") + ["--save-every", "4", "--peer-timeout", "20"]
    procs = _launch(d, "960", args, 2, {"FT_INJECT_FAULT": f"1:3:{phase}"})
    rcs, waited = _wait_all(procs, timeout=240)
    logs = _logs(d, "960", 2)
    assert rcs == [0, 0], logs
    assert _saved_steps(logs) == [saved, saved], logs
    assert not any("Checkpoint written" in o for o in logs), logs  # the periodic save never started
    assert not any("Lost a peer rank" in o for o in logs), logs
    _assert_same_state(_load(d, "960"), _reference_at(d, "zero1", 2, saved))


@pytest.mark.parametrize("world", [2, 4])
def test_sigkilled_rank_zero1_resumes_from_periodic_save(tmp_path, world):
    """ZeRO-1 (the default DP mode) cannot write a checkpoint without the dead rank's optimizer
    shards; the periodic saves (on by default under DP) are the recovery point. A rank is
    SIGKILLed after a periodic save became durable: the survivors exit non-zero within the
    peer timeout naming that checkpoint, and a job resumed from it reaches the same state,
    bit for bit, as an uninterrupted run."""
    d = str(tmp_path)
    write_fake_sbatch(d)
    args = _base(d, "zero1", steps=10000) + ["--save-every", "4", "--peer-timeout", "20"]
    procs = _launch(d, "970", args, world, {"FT_INJECT_FAULT": "1:10:kill"})
    try:
        assert procs[1].wait(timeout=240) == -signal.SIGKILL
        t_kill = time.time()
        rcs = [p.wait(timeout=60) for i, p in enumerate(procs) if i != 1]
        waited = time.time() - t_kill
    finally:
        for p in procs:
            kill_group(p)
    logs = _logs(d, "970", world)
    survivors = [o for i, o in enumerate(logs) if i != 1]
    assert rcs == [1] * (world - 1), logs
    assert waited < 30, waited
    assert all("Lost a peer rank" in o for o in survivors), survivors
    assert _saved_steps(survivors) == [], survivors  # no new file without the lost shards
    durable = {int(m.group(1)) for m in (re.search(r"Last durable checkpoint: .* at step (\d+)", o)
                                         for o in survivors) if m}
    assert len(durable) == 1 and durable <= {4, 8}, survivors
    n = durable.pop()
    assert _load(d, "970")["training_step"] == n

    # resume from the periodic checkpoint to step 14 and compare with an uninterrupted run
    resume = _base(d, "zero1", steps=16) + ["--checkpoint-id", "970", "--raise-error", "--error-step", "14"]
    rcs, _ = _wait_all(_launch(d, "971", resume, world))
    logs = _logs(d, "971", world)
    assert rcs == [0] * world, logs
    assert f"Resuming training from training_step {n}" in logs[0], logs[0]
    assert _saved_steps(logs) == [14] * world, logs
    _assert_same_state(_load(d, "971"), _reference_at(d, "zero1", world, 14, ["--training-steps", "16"]))
