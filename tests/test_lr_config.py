"""LR schedule (reference utils.py:32-56) and CLI surface (reference utils.py:112-203)."""
import torch

from fault_tolerant_llm_training_amd.utils.config import get_args
from fault_tolerant_llm_training_amd.utils.lr import build_lr_scheduler, linear_warmup_constant


def test_warmup_then_constant():
    assert linear_warmup_constant(10, 0) == 1 / 11
    assert linear_warmup_constant(10, 9) == 10 / 11
    assert linear_warmup_constant(10, 10) == 1.0
    assert linear_warmup_constant(10, 10_000) == 1.0  # constant, not decaying


def test_lambdalr_matches_reference_sequence():
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=5e-5)
    s = build_lr_scheduler(opt, 100)
    lrs = []
    for _ in range(105):
        lrs.append(opt.param_groups[0]["lr"])
        opt.step()
        s.step()
    assert abs(lrs[0] - 5e-5 / 101) < 1e-15
    assert abs(lrs[99] - 5e-5 * 100 / 101) < 1e-15
    assert lrs[100] == lrs[104] == 5e-5
    sd = s.state_dict()
    s2 = build_lr_scheduler(torch.optim.SGD([p], lr=5e-5), 100)
    s2.load_state_dict(sd)
    assert s2.last_epoch == s.last_epoch


def test_reference_flags_and_defaults(monkeypatch):
    monkeypatch.setenv("WORKDIR", "/w")
    a = get_args([])
    assert a.dataset == "/capstor/store/cscs/ethz/large-sc/datasets/train_data.parquet"
    assert a.checkpoint_path == "/w/checkpoints"
    assert a.checkpoint_id == ""
    assert a.tokenizer_name_or_path == "unsloth/Mistral-Nemo-Base-2407-bnb-4bit"
    assert (a.sequence_length, a.batch_size, a.learning_rate) == (4096, 1, 1e-5)
    assert (a.lr_warmup_steps, a.training_steps, a.logging_frequency) == (10, 1000, 5)
    assert (a.grad_max_norm, a.model_dtype, a.error_step) == (1, "bf16", 100)
    assert not (a.fused_optimizer or a.compile or a.raise_error)
    b = get_args(["--sequence-length", "2048", "--raise-error", "--error-step", "600", "--checkpoint-id", "444664",
                  "--fused-optimizer", "--compile"])
    assert (b.sequence_length, b.raise_error, b.error_step, b.checkpoint_id) == (2048, True, 600, "444664")
