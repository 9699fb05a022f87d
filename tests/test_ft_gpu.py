"""The fault-tolerance flow of train.py on the MI355X (reference train.py:89-129, utils.py:65-97).

On the GPU the whole production path runs: HIP kernels, the dW side stream, the pipelined
optimizer, the asynchronous native checkpoint engine (HBM snapshot -> pinned D2H -> O_DIRECT
zip writer) and the pinned-ring restore. Checked here:

* an injected error saves (no resubmit) and a resumed job continues from the saved step;
* the resumed run ends bit-identical to an uninterrupted run (parameters and AdamW moments);
* SIGUSR1 saves and resubmits through ``sbatch`` with the job id (reference utils.py:81-85).
"""
import os
import shutil
import signal

import pytest
import torch

from helpers import kill_group, run_train, sbatch_calls, start_train, wait_for_log, write_fake_sbatch

pytestmark = pytest.mark.gpu

GPU = ["--device", "cuda", "--model", "tiny", "--synthetic-data", "--vocab-size", "1024", "--sequence-length", "256",
       "--batch-size", "2", "--learning-rate", "1e-3", "--lr-warmup-steps", "3", "--logging-frequency", "5"]


def _load(d, job):
    return torch.load(os.path.join(d, "ck", f"checkpoint_{job}.ckpt"), map_location="cpu", weights_only=True)


def test_gpu_error_save_resume_bit_exact(tmp_path):
    d = str(tmp_path)
    write_fake_sbatch(d)
    base = GPU + ["--checkpoint-path", os.path.join(d, "ck"), "--training-steps", "41"]
    rc, out = run_train(d, "700", base + ["--raise-error", "--error-step", "40"], timeout=240)
    assert rc == 0 and "Checkpoint saved at step 40" in out, out[-3000:]
    rc, out = run_train(d, "701", base + ["--raise-error", "--error-step", "15"], timeout=240)
    assert rc == 0 and "Checkpoint saved at step 15" in out, out[-3000:]
    assert not sbatch_calls(d)  # errors do not resubmit
    rc, out = run_train(d, "702", base + ["--raise-error", "--error-step", "40", "--checkpoint-id", "701"],
                        timeout=240)
    assert rc == 0 and "Resuming training from training_step 15" in out, out[-3000:]
    a, c = _load(d, 700), _load(d, 702)
    assert a["training_step"] == c["training_step"] == 40
    for k in a["model"]:
        assert torch.equal(a["model"][k], c["model"][k]), k
    for i in a["optimizer"]["state"]:
        assert torch.equal(a["optimizer"]["state"][i]["exp_avg"], c["optimizer"]["state"][i]["exp_avg"])
        assert torch.equal(a["optimizer"]["state"][i]["exp_avg_sq"], c["optimizer"]["state"][i]["exp_avg_sq"])


def test_gpu_sigusr1_saves_and_resubmits(tmp_path):
    d = str(tmp_path)
    write_fake_sbatch(d)
    args = GPU + ["--checkpoint-path", os.path.join(d, "ck"), "--training-steps", "100000"]
    p = start_train(d, "710", args)
    try:
        assert wait_for_log(p._log_path, "Training step: 10 |", timeout=180), open(p._log_path).read()[-3000:]
        os.kill(p.pid, signal.SIGUSR1)
        assert p.wait(timeout=180) == 0
    finally:
        kill_group(p)
    out = open(p._log_path).read()
    assert "[EXIT HANDLER] Job timed out, saving checkpoint." in out, out[-3000:]
    assert "Checkpoint saved at step" in out and "sbatch requeued" in out, out[-3000:]
    calls = sbatch_calls(d)
    assert calls and calls[0][-1] == "710", calls
    c = _load(d, 710)
    assert c["training_step"] >= 10


def _same(a, b):
    assert a["training_step"] == b["training_step"]
    for k in a["model"]:
        assert torch.equal(a["model"][k], b["model"][k]), k
    for i in a["optimizer"]["state"]:
        for key in ("exp_avg", "exp_avg_sq", "step"):
            assert torch.equal(a["optimizer"]["state"][i][key], b["optimizer"]["state"][i][key]), (i, key)
    assert a["lr_scheduler"] == b["lr_scheduler"]
    assert a["data_loader"] == b["data_loader"]


def test_gpu_async_periodic_checkpoint_equals_blocking_and_resumes_bit_exact(tmp_path):
    """--save-every on the production path (HBM snapshot overlapping the next steps, pipelined
    optimizer, dW side stream) writes the same bytes as a blocking save, and resumes bit-exactly."""
    d = str(tmp_path)
    write_fake_sbatch(d)
    base = GPU + ["--checkpoint-path", os.path.join(d, "ck")]
    rc, out = run_train(d, "720", base + ["--training-steps", "10", "--save-every", "4"], timeout=240)
    assert rc == 0 and "Checkpoint written" in out, out[-3000:]
    rc, out = run_train(d, "721", base + ["--training-steps", "10", "--save-every", "4", "--no-async-checkpoint"],
                        timeout=240)
    assert rc == 0, out[-3000:]
    a, b = _load(d, 720), _load(d, 721)
    assert a["training_step"] == 8  # the last periodic save (saves at 4 and 8)
    _same(a, b)
    rc, out = run_train(d, "722", base + ["--training-steps", "20", "--raise-error", "--error-step", "13",
                                          "--checkpoint-id", "720"], timeout=240)
    assert rc == 0 and "Resuming training from training_step 8" in out and "Checkpoint saved at step 13" in out
    rc, out = run_train(d, "723", base + ["--training-steps", "20", "--raise-error", "--error-step", "13"],
                        timeout=240)
    assert rc == 0 and "Checkpoint saved at step 13" in out, out[-3000:]
    _same(_load(d, 722), _load(d, 723))


def test_gpu_nonfinite_gradient_saves_state_before_the_bad_step(tmp_path):
    """Non-finite gradient norm (reference utils.py:61 error_if_nonfinite -> train.py:121-129): the
    device-side sticky guard skips the update, the host finds the bad step two steps later and
    rolls back to it; the file equals an injected-error save at that step."""
    d = str(tmp_path)
    write_fake_sbatch(d)
    base = GPU[:-6] + ["--learning-rate", "1e30", "--lr-warmup-steps", "3", "--logging-frequency", "1",
                       "--checkpoint-path", os.path.join(d, "ck"), "--training-steps", "30"]
    rc, out = run_train(d, "730", base, timeout=240)
    assert rc == 0 and "is non-finite at optimizer step" in out, out[-3000:]
    import re

    n = int(re.search(r"Checkpoint saved at step (\d+)", out).group(1))
    assert 0 < n < 30
    rc, out2 = run_train(d, "731", base + ["--raise-error", "--error-step", str(n)], timeout=240)
    assert rc == 0 and f"Checkpoint saved at step {n}" in out2, out2[-3000:]
    _same(_load(d, 730), _load(d, 731))


@pytest.mark.timeout(900)
def test_gpu_llama8b_iterable_error_resume_bit_exact(tmp_path):
    """BASELINE config 4 at its scale: Llama-3-8B, seq 2048, the packing IterableParquetDataset
    (reference dataset.py:56-101, byte tokenizer on a generated parquet; train.py:36-39's
    fast-forward is the dataset's mid-shard state here). An injected error at step 5 saves the
    48 GB state; the resumed job runs to step 12 and must end with exactly the parameters, AdamW
    moments, optimizer step and data-loader position of an uninterrupted run to step 12 (bit-level
    digests, --state-digest: one checkpoint on disk instead of three)."""
    import re

    from helpers import make_parquet

    d = str(tmp_path)
    write_fake_sbatch(d)
    pq = os.path.join(d, "train.parquet")
    make_parquet(pq, n_docs=5000, seed=3)
    base = ["--device", "cuda", "--model", "llama3-8b", "--dataset", pq, "--iterable-dataset",
            "--tokenizer-name-or-path", "byte", "--vocab-size", "131072", "--sequence-length", "2048",
            "--batch-size", "1", "--learning-rate", "5e-5", "--lr-warmup-steps", "100", "--logging-frequency", "4",
            "--checkpoint-path", os.path.join(d, "ck"), "--training-steps", "12", "--state-digest"]

    def digest(out):
        m = re.search(r"State digest at step (\d+): (.*)", out)
        assert m, out[-3000:]
        return int(m.group(1)), m.group(2).strip()

    try:
        rc, out = run_train(d, "790", base, timeout=600)
        assert rc == 0 and "Training completed" in out, out[-3000:]
        ref = digest(out)
        assert ref[0] == 12
        rc, out = run_train(d, "791", base + ["--raise-error", "--error-step", "5"], timeout=600)
        assert rc == 0 and "Checkpoint saved at step 5" in out, out[-3000:]
        saved = re.search(r"State digest at step 5 \(saved\): (.*)", out)
        rc, out = run_train(d, "792", base + ["--checkpoint-id", "791"], timeout=600)
        assert rc == 0 and "Resuming training from training_step 5" in out, out[-3000:]
        assert "Data loader position restored" in out
        resumed = re.search(r"State digest at step 5 \(resumed\): (.*)", out)
        assert saved and resumed and saved.group(1).strip() == resumed.group(1).strip()
        assert digest(out) == ref
    finally:  # the 48 GB checkpoint: pytest keeps tmp dirs, and later jobs on the box need the disk
        shutil.rmtree(os.path.join(d, "ck"), ignore_errors=True)
