"""Whole-step HIP-graph replay (graphs.GraphedStep) == eager steps, bit for bit, on the MI355X.

The graph holds the optimizer step of the previous backward plus the next forward/backward
(bucket hooks, dW side stream, per-layer ParamGate waits as graph edges); lr and the AdamW
bias corrections come from a device buffer staged before each replay."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(preset, V, S):
    from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for
    from fault_tolerant_llm_training_amd.optim.adamw import FlatAdamW
    from fault_tolerant_llm_training_amd.parallel.ddp import GradReducer
    from fault_tolerant_llm_training_amd.utils.lr import build_lr_scheduler

    a = model_args_for(preset, vocab_size=V, seq_len=S)
    m = build_model(a, "cuda", torch.bfloat16, seed=3)
    red = GradReducer(m.flat, m.sinks_in_backward_order(), bucket_mb=1.0)
    opt = FlatAdamW(m.parameters(), m.flat, lr=3e-3, max_grad_norm=1.0, reducer=red)
    m.gate = opt.gate
    sched = build_lr_scheduler(opt, 4)  # warmup: the lr changes every replay
    return m, red, opt, sched


@pytest.mark.parametrize("preset,V,S", [("tiny", 1024, 256), ("gpt2-small", 8192, 512)])
def test_graphed_steps_bitwise_equal_eager(preset, V, S):
    from fault_tolerant_llm_training_amd.data.synthetic import SyntheticTokens
    from fault_tolerant_llm_training_amd.graphs import GraphedStep

    data = SyntheticTokens(V, S, seed=11)
    inv = torch.full((1,), 1.0 / (2 * S), device="cuda")
    batches = [data.batch(i, 2) for i in range(7)]

    m, red, opt, sched = _setup(preset, V, S)
    losses_e = []
    for tok, lab in batches:
        loss = m(tok.cuda(), lab.cuda(), inv)
        loss.backward()
        red.finish()
        opt.step()
        sched.step()
        losses_e.append(loss.item())
    pe, me, ve = m.flat.params.clone(), opt.exp_avg.clone(), opt.exp_avg_sq.clone()

    m2, red2, opt2, sched2 = _setup(preset, V, S)

    def fwd_bwd(tok, lab):
        loss = m2(tok, lab, inv)
        loss.backward()
        red2.finish()
        return loss

    gs = GraphedStep(m2, red2, opt2, sched2, fwd_bwd)
    losses_g = []
    for tok, lab in batches[:2]:  # eager warmup steps
        loss = fwd_bwd(tok.cuda(), lab.cuda())
        opt2.step()
        sched2.step()
        losses_g.append(loss.item())
    losses_g.append(gs.prime(*batches[2]).item())
    for tok, lab in batches[3:]:
        losses_g.append(gs.step(tok, lab).item())
    gs.finish()
    torch.cuda.synchronize()
    assert losses_g == losses_e
    assert opt2.step_count == opt.step_count == 7
    assert torch.equal(m2.flat.params, pe)
    assert torch.equal(opt2.exp_avg, me) and torch.equal(opt2.exp_avg_sq, ve)
    assert opt2.check_finite(block=True) is not None


def test_train_py_hip_graph_matches_eager_and_saves(tmp_path):
    """train.py --hip-graph: same checkpoint as the eager run at an injected error (the pending
    optimizer step is completed before the save), and a periodic save re-primes the graph."""
    import os

    from helpers import run_train, write_fake_sbatch

    d = str(tmp_path)
    write_fake_sbatch(d)
    base = ["--device", "cuda", "--model", "tiny", "--synthetic-data", "--vocab-size", "1024",
            "--sequence-length", "256", "--batch-size", "2", "--learning-rate", "1e-3", "--lr-warmup-steps", "3",
            "--logging-frequency", "1", "--checkpoint-path", os.path.join(d, "ck"), "--training-steps", "30",
            "--raise-error", "--error-step", "17"]
    rc, out = run_train(d, "760", base, timeout=240)
    assert rc == 0 and "Checkpoint saved at step 17" in out, out[-3000:]
    rc, out = run_train(d, "761", base + ["--hip-graph", "--save-every", "8"], timeout=240)
    assert rc == 0 and "Checkpoint saved at step 17" in out and "HIP graph" in out, out[-3000:]
    load = lambda j: torch.load(os.path.join(d, "ck", f"checkpoint_{j}.ckpt"), map_location="cpu",  # noqa: E731
                                weights_only=True)
    a, b = load(760), load(761)
    assert a["training_step"] == b["training_step"] == 17
    for k in a["model"]:
        assert torch.equal(a["model"][k], b["model"][k]), k
    for i in a["optimizer"]["state"]:
        assert torch.equal(a["optimizer"]["state"][i]["exp_avg_sq"], b["optimizer"]["state"][i]["exp_avg_sq"])
    assert a["lr_scheduler"] == b["lr_scheduler"]
    # the logged losses agree too
    import re

    la = re.findall(r"Training step: (\d+) \| Loss: ([0-9.]+)", out)
    assert len(la) >= 15


def test_train_py_compile_is_the_hip_graph_and_resumes_bit_exact(tmp_path):
    """train.py --compile (reference train.py:61-63) on one GPU = the whole-step HIP graph: the
    reference's log line, graph replays, an injected error saves, the resumed --compile job ends
    bit-identical (params, both moments, scheduler) to an uninterrupted eager run."""
    import os

    from helpers import run_train, write_fake_sbatch

    d = str(tmp_path)
    write_fake_sbatch(d)
    ck = os.path.join(d, "ck")
    base = ["--device", "cuda", "--model", "tiny", "--synthetic-data", "--vocab-size", "1024",
            "--sequence-length", "256", "--batch-size", "2", "--learning-rate", "1e-3", "--lr-warmup-steps", "3",
            "--logging-frequency", "5", "--checkpoint-path", ck, "--training-steps", "40", "--raise-error"]
    rc, out = run_train(d, "780", base + ["--error-step", "30"], timeout=240)  # eager reference
    assert rc == 0 and "Checkpoint saved at step 30" in out, out[-3000:]
    rc, out = run_train(d, "781", base + ["--compile", "--error-step", "17"], timeout=240)
    assert rc == 0 and "Using `torch.compile`" in out and "HIP graph" in out, out[-3000:]
    assert "Checkpoint saved at step 17" in out, out[-3000:]
    rc, out = run_train(d, "782", base + ["--compile", "--error-step", "30", "--checkpoint-id", "781"], timeout=240)
    assert rc == 0 and "Resuming training from training_step 17" in out and "HIP graph" in out, out[-3000:]
    assert "Checkpoint saved at step 30" in out, out[-3000:]
    load = lambda j: torch.load(os.path.join(ck, f"checkpoint_{j}.ckpt"), map_location="cpu",  # noqa: E731
                                weights_only=True)
    a, b = load(780), load(782)
    assert a["training_step"] == b["training_step"] == 30
    for k in a["model"]:
        assert torch.equal(a["model"][k], b["model"][k]), k
    for i in a["optimizer"]["state"]:
        for key in ("exp_avg", "exp_avg_sq", "step"):
            assert torch.equal(a["optimizer"]["state"][i][key], b["optimizer"]["state"][i][key]), (i, key)
    assert a["lr_scheduler"] == b["lr_scheduler"]


def test_train_py_compile_fp64_runs_eager(tmp_path):
    """--compile --model-dtype fp64 (both accepted by the reference, train.py:61-63, utils.py:14-19):
    the fp64 composed path syncs with the host inside the step, so no HIP graph is captured; the
    run trains eagerly to completion with the reference's log line."""
    import os

    from helpers import run_train, write_fake_sbatch

    d = str(tmp_path)
    write_fake_sbatch(d)
    args = ["--device", "cuda", "--model", "tiny", "--synthetic-data", "--vocab-size", "256",
            "--sequence-length", "64", "--batch-size", "1", "--model-dtype", "fp64", "--compile",
            "--logging-frequency", "2", "--checkpoint-path", os.path.join(d, "ck"), "--training-steps", "4"]
    rc, out = run_train(d, "790", args, timeout=240)
    assert rc == 0 and "Using `torch.compile`" in out and "not applied" in out, out[-3000:]
    assert "HIP graph:" not in out and "Training completed" in out, out[-3000:]
