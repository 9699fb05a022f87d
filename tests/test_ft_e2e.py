"""End-to-end fault tolerance on the CPU: real signals to a real train.py process.

* SIGUSR1 → "[EXIT HANDLER] Job timed out" → checkpoint → ``sbatch $WORKDIR/train.sh $JOBID``
  (fake sbatch) → resumed job continues from the saved step (reference logs
  output_444664.out:93-106 → output_444671.out:5-13);
* SIGTERM → "Job cancelled", no checkpoint (output_444691.out:58-63);
* ``--raise-error --error-step N`` → save at N, no resubmit (output_444671.out:46-48);
* resume equivalence: interrupted + resumed runs end bit-identical to an
  uninterrupted run (model, AdamW moments, LR schedule, data position) — the
  "zero steps lost" acceptance test, for every data source.
"""
import os
import re
import signal

import pytest
import torch

from helpers import TINY, kill_group, make_parquet, run_train, sbatch_calls, start_train, wait_for_log, \
    write_fake_sbatch

pytestmark = pytest.mark.slow

SYN = TINY + ["--synthetic-data", "--vocab-size", "256"]


def _ckpt(d, job):
    return os.path.join(d, "ck", f"checkpoint_{job}.ckpt")


def _common(d):
    return ["--checkpoint-path", os.path.join(d, "ck")]


def test_sigusr1_saves_resubmits_and_resumes(tmp_path):
    d = str(tmp_path)
    write_fake_sbatch(d)
    p = start_train(d, "1001", SYN + _common(d) + ["--training-steps", "1000000"])
    try:
        assert wait_for_log(p._log_path, "Training step: 5 |"), open(p._log_path).read()
        os.kill(p.pid, signal.SIGUSR1)
        assert p.wait(timeout=120) == 0
    finally:
        kill_group(p)
    out = open(p._log_path).read()
    assert "[EXIT HANDLER] Job timed out, saving checkpoint." in out
    m = re.search(r"\[EXIT HANDLER\] Checkpoint saved at step (\d+)", out)
    assert m, out
    saved_step = int(m.group(1))
    assert "[EXIT HANDLER] sbatch requeued, new job will load the last checkpoint" in out
    assert "Submitted batch job 424242" in out
    assert sbatch_calls(d) == [[os.path.join(d, "train.sh"), "1001"]]
    c = torch.load(_ckpt(d, "1001"), map_location="cpu", weights_only=True)
    assert c["training_step"] == saved_step
    assert c["lr_scheduler"]["last_epoch"] == saved_step  # no torn step
    # the resubmitted job: train.sh passes $1 as --checkpoint-id
    rc, out2 = run_train(d, "1002", SYN + _common(d) + ["--training-steps", str(saved_step + 3),
                                                        "--checkpoint-id", "1001"])
    assert rc == 0, out2
    for line in ("Loading checkpoint from", "Model loaded from checkpoint", "Optimizer loaded from checkpoint",
                 "LR Scheduler loaded from checkpoint", f"Resuming training from training_step {saved_step}",
                 "Training completed"):
        assert line in out2, (line, out2)


def test_sigterm_cancels_without_checkpoint(tmp_path):
    d = str(tmp_path)
    write_fake_sbatch(d)
    p = start_train(d, "2001", SYN + _common(d) + ["--training-steps", "1000000"])
    try:
        assert wait_for_log(p._log_path, "Training step: 1 |")
        os.kill(p.pid, signal.SIGTERM)
        assert p.wait(timeout=120) == 0
    finally:
        kill_group(p)
    out = open(p._log_path).read()
    assert "[EXIT HANDLER] Job cancelled, terminating." in out
    assert "Checkpoint saved" not in out
    assert not os.path.exists(_ckpt(d, "2001"))
    assert sbatch_calls(d) == []


def test_signal_during_setup_is_deferred_to_first_boundary(tmp_path):
    """The reference installs its handler after setup (train.py:89-90): an early USR1 killed it."""
    d = str(tmp_path)
    write_fake_sbatch(d)
    p = start_train(d, "3001", SYN + _common(d) + ["--training-steps", "1000000"])
    try:
        assert wait_for_log(p._log_path, "Setting up DataLoaders")
        os.kill(p.pid, signal.SIGUSR1)
        assert p.wait(timeout=120) == 0
    finally:
        kill_group(p)
    out = open(p._log_path).read()
    # the first step boundary is the vote before step 0: nothing has been computed yet
    assert "[EXIT HANDLER] Checkpoint saved at step 0" in out, out


def test_injected_error_saves_without_resubmit(tmp_path):
    d = str(tmp_path)
    write_fake_sbatch(d)
    rc, out = run_train(d, "4001", SYN + _common(d) + ["--training-steps", "50", "--raise-error",
                                                       "--error-step", "7"])
    assert rc == 0
    assert "[EXIT HANDLER] Error during training encountered, saving checkpoint." in out
    assert "[EXIT HANDLER] Checkpoint saved at step 7" in out
    assert sbatch_calls(d) == []
    assert "Training step: 5 | Loss:" in out and "Training step: 7 |" not in out


def _final_state(path):
    c = torch.load(path, map_location="cpu", weights_only=True)
    return c


def _assert_same_state(a, b):
    assert a["training_step"] == b["training_step"]
    for k in a["model"]:
        assert torch.equal(a["model"][k], b["model"][k]), k
    for i in a["optimizer"]["state"]:
        for f in ("exp_avg", "exp_avg_sq", "step"):
            assert torch.equal(a["optimizer"]["state"][i][f], b["optimizer"]["state"][i][f]), (i, f)
    assert a["lr_scheduler"] == b["lr_scheduler"]
    assert a["data_loader"] == b["data_loader"]


@pytest.mark.parametrize("source", ["synthetic", "parquet", "iterable"])
def test_resume_is_bit_exact(tmp_path, source):
    d = str(tmp_path)
    write_fake_sbatch(d)
    if source == "synthetic":
        base = SYN
    else:
        pq = os.path.join(d, "data.parquet")
        make_parquet(pq, n_docs=30)
        base = TINY + ["--dataset", pq, "--tokenizer-name-or-path", "byte"]
        if source == "iterable":
            base = base + ["--iterable-dataset"]
    base = base + _common(d) + ["--training-steps", "13", "--lr-warmup-steps", "4"]
    end = ["--raise-error", "--error-step", "12"]
    # uninterrupted reference run, state captured at step 12
    rc, out = run_train(d, "10", base + end)
    assert rc == 0 and "Checkpoint saved at step 12" in out, out
    # interrupted at 5, resumed, state captured at 12
    rc, out = run_train(d, "20", base + ["--raise-error", "--error-step", "5"])
    assert rc == 0 and "Checkpoint saved at step 5" in out
    rc, out = run_train(d, "30", base + end + ["--checkpoint-id", "20"])
    assert rc == 0 and "Resuming training from training_step 5" in out, out
    _assert_same_state(_final_state(_ckpt(d, "10")), _final_state(_ckpt(d, "30")))


def _digest(out):
    m = re.search(r"State digest at step (\d+): (.*)", out)
    assert m, out[-3000:]
    return int(m.group(1)), m.group(2).strip()


def test_state_digest_resume_equivalence_iterable(tmp_path):
    """--state-digest (the full-scale form of the check above: no second checkpoint on disk): the
    uninterrupted and the interrupted-then-resumed iterable-dataset runs log identical digests of
    parameters, moments, optimizer step and data-loader position; a different run does not."""
    d = str(tmp_path)
    write_fake_sbatch(d)
    pq = os.path.join(d, "data.parquet")
    make_parquet(pq, n_docs=30)
    base = (TINY + ["--dataset", pq, "--tokenizer-name-or-path", "byte", "--iterable-dataset", "--state-digest"]
            + _common(d) + ["--training-steps", "11", "--lr-warmup-steps", "4"])
    rc, out = run_train(d, "40", base)
    assert rc == 0 and "Training completed" in out, out[-3000:]
    ref = _digest(out)
    rc, out = run_train(d, "41", base + ["--raise-error", "--error-step", "6"])
    assert rc == 0 and "Checkpoint saved at step 6" in out
    saved = re.search(r"State digest at step 6 \(saved\): (.*)", out)
    assert saved, out[-3000:]
    rc, out = run_train(d, "42", base + ["--checkpoint-id", "41"])
    assert rc == 0 and "Resuming training from training_step 6" in out, out[-3000:]
    # the state the exit handler saved is the state the next job resumes from, bit for bit
    resumed = re.search(r"State digest at step 6 \(resumed\): (.*)", out)
    assert resumed and resumed.group(1).strip() == saved.group(1).strip(), (saved, resumed)
    assert _digest(out) == ref and ref[0] == 11
    rc, out = run_train(d, "43", base + ["--seed", "99"])
    assert rc == 0 and _digest(out)[1] != ref[1]


def test_sigusr1_preempt_resume_loses_zero_steps(tmp_path):
    """Preempt at an arbitrary moment with SIGUSR1, resume, compare with the uninterrupted run."""
    d = str(tmp_path)
    write_fake_sbatch(d)
    base = SYN + _common(d) + ["--training-steps", "41", "--lr-warmup-steps", "4"]
    end = ["--raise-error", "--error-step", "40"]
    rc, out = run_train(d, "50", base + end)
    assert rc == 0
    p = start_train(d, "60", base + end)
    try:
        assert wait_for_log(p._log_path, "Training step: 10 |")
        os.kill(p.pid, signal.SIGUSR1)
        assert p.wait(timeout=120) == 0
    finally:
        kill_group(p)
    out = open(p._log_path).read()
    m = re.search(r"Checkpoint saved at step (\d+)", out)
    assert m and "Job timed out" in out, out
    assert int(m.group(1)) < 40
    rc, out = run_train(d, "70", base + end + ["--checkpoint-id", "60"])
    assert rc == 0, out
    _assert_same_state(_final_state(_ckpt(d, "50")), _final_state(_ckpt(d, "70")))


def test_sigusr1_state_digest_saved_equals_resumed_iterable(tmp_path):
    """SIGUSR1 mid-run on the iterable dataset (the loader has usually fetched the next batch when
    the signal is acted on): the digest logged at the exit-handler save, loader position included,
    equals the one logged after the next job resumed from that checkpoint."""
    d = str(tmp_path)
    write_fake_sbatch(d)
    pq = os.path.join(d, "data.parquet")
    make_parquet(pq, n_docs=60)
    base = (TINY + ["--dataset", pq, "--tokenizer-name-or-path", "byte", "--iterable-dataset", "--state-digest"]
            + _common(d) + ["--training-steps", "100000", "--lr-warmup-steps", "4"])
    p = start_train(d, "61", base)
    try:
        assert wait_for_log(p._log_path, "Training step: 10 |")
        os.kill(p.pid, signal.SIGUSR1)
        assert p.wait(timeout=120) == 0
    finally:
        kill_group(p)
    out = open(p._log_path).read()
    saved = re.search(r"State digest at step (\d+) \(saved\): (.*)", out)
    assert saved and "Job timed out" in out, out[-3000:]
    rc, out = run_train(d, "62", base[:-4] + ["--training-steps", str(int(saved.group(1)) + 1), "--lr-warmup-steps",
                                              "4", "--checkpoint-id", "61"])
    assert rc == 0, out[-3000:]
    resumed = re.search(r"State digest at step (\d+) \(resumed\): (.*)", out)
    assert resumed and resumed.groups() == saved.groups(), (saved.groups(), resumed and resumed.groups())


def test_periodic_async_checkpoint(tmp_path):
    d = str(tmp_path)
    rc, out = run_train(d, "80", SYN + _common(d) + ["--training-steps", "9", "--save-every", "4"])
    assert rc == 0 and "Training completed" in out
    assert "Checkpoint written:" in out
    c = torch.load(_ckpt(d, "80"), map_location="cpu", weights_only=True)
    assert c["training_step"] == 8
