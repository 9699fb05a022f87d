"""GEMM routing table per preset and dtype (ops/routing.py: routing_table evaluates the same
predicates the autograd functions use, on shape/dtype specs: no GPU needed). Pins which kernel
each product of the step takes, so a routing change is a visible test change:

* Llama-3-8B bf16 / fp16: every product on the hand-written w4 kernel -- none on hipBLASLt (the
  deep-reduction dX products with a K split);
* fp32 models: every product on the hand-written fp32 MFMA kernel (gemm_f32.hip); CPU tensors:
  the composed path;
* GPT-2-sized presets at one sequence: every product on w4 too (round 6: K splits for the small
  grids, a tail tile for V % 256), none on hipBLASLt.
"""
import pytest
import torch

from fault_tolerant_llm_training_amd.models.llama import model_args_for
from fault_tolerant_llm_training_amd.ops import functional as Fx
from fault_tolerant_llm_training_amd.ops.routing import routing_table

PRODUCTS = ["qkv fwd", "qkv dX", "qkv dW", "wo fwd", "wo dX", "wo dW", "w13 fwd", "w2 dX", "w13 dX", "w13 dW",
            "w2 fwd", "w2 dW", "head fwd", "head dX", "head dW"]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_llama8b_every_product_on_w4(dtype):
    t = routing_table(model_args_for("llama3-8b", vocab_size=131072, seq_len=2048), dtype)
    assert sorted(t) == sorted(PRODUCTS)
    assert t == {
        "qkv fwd": "w4 qkv+rope", "qkv dX": "w4 256 x2", "qkv dW": "w4 256",
        "wo fwd": "w4 128", "wo dX": "w4 128", "wo dW": "w4 256",
        "w13 fwd": "w4 swiglu", "w2 dX": "w4 swiglu-bwd", "w13 dX": "w4 256 x2", "w13 dW": "w4 256",
        "w2 fwd": "w4 256 x2", "w2 dW": "w4 224",
        "head fwd": "w4 256", "head dX": "w4 256 x2", "head dW": "w4 256",
    }


@pytest.mark.parametrize("preset", ["llama3-8b", "gpt2-small", "gpt2-medium"])
def test_fp32_takes_the_f32_mfma_gemm_and_cpu_the_composed_path(preset, monkeypatch):
    """fp32 models (reference utils.py:14-19): every product of the layer and the LM head on the fp32
    MFMA kernel (round 6; before: hipBLASLt); set_f32_mfma(False) / FT_F32_MFMA=0 restores hipBLASLt."""
    a = model_args_for(preset, vocab_size=50304 if preset != "llama3-8b" else 131072, seq_len=2048)
    assert set(routing_table(a, torch.float32).values()) == {"f32 mfma"}
    assert set(routing_table(a, torch.bfloat16, cuda=False).values()) == {"hipBLASLt"}
    assert set(routing_table(a, torch.float64).values()) == {"hipBLASLt"}
    monkeypatch.setattr(Fx, "_F32_MFMA", False)
    assert set(routing_table(a, torch.float32).values()) == {"hipBLASLt"}


@pytest.mark.parametrize("preset,vocab", [("gpt2-small", 50304), ("gpt2-small", 131072),
                                          ("gpt2-medium", 50304), ("gpt2-medium", 131072)])
def test_gpt2_routes(preset, vocab):
    """Round 6: no GPT-2 product on hipBLASLt. The 18-96-tile weight gradients take a K split (the
    dW layout splits its 128-wide tile), the 2048-3072-deep forward / dX products too, the FFN runs
    fused (SwiGLU in the w1|w3 epilogue, its backward in the w2 dX epilogue), the LM-head dW at the
    padded V = 50304 a tail tile, the V = 131072 logits the 256-wide tile (K = 768 / 1024)."""
    t = routing_table(model_args_for(preset, vocab_size=vocab, seq_len=2048), torch.bfloat16)
    assert sorted(t) == sorted(PRODUCTS)
    assert "hipBLASLt" not in t.values(), t
    assert t["head dX"].startswith("w4") and " x" in t["head dX"]
    assert t["wo fwd"] == t["wo dX"] == "w4 128"
    for k in ("qkv dW", "wo dW", "w2 dW", "w2 fwd", "qkv dX"):
        assert " x" in t[k], (k, t[k])
    assert t["w13 fwd"] == "w4 swiglu" and t["w2 dX"] == "w4 swiglu-bwd"
    assert t["head dW"].startswith("w4")
    if vocab == 131072:
        assert t["head fwd"] == "w4 256"


def test_gpt2_round5_routing_knob(monkeypatch):
    """set_w4_small(False) (FT_W4_SMALL=0): the round-5 routing of the small products (A/B)."""
    monkeypatch.setattr(Fx, "_W4_SMALL", False)
    t = routing_table(model_args_for("gpt2-small", vocab_size=50304, seq_len=2048), torch.bfloat16)
    assert t["wo dW"] == t["head dW"] == "hipBLASLt" and t["wo fwd"] == "w4 128"


def test_blas_only_knob(monkeypatch):
    monkeypatch.setattr(Fx, "_BLAS_ONLY", True)
    from fault_tolerant_llm_training_amd.ops import attention as A

    t = routing_table(model_args_for("llama3-8b", vocab_size=131072, seq_len=2048), torch.bfloat16)
    assert set(t.values()) == {"hipBLASLt"}
    assert A._qkv_rope_ok is not None


def test_fp32_model_logs_its_gemm_kernel_once(tmp_path):
    """--model-dtype fp32 (reference utils.py:14-19): the w4 GEMM is 16-bit, so the GEMMs of an fp32
    model take the fp32 MFMA kernel (hipBLASLt where K % 32 != 0) -- logged once at startup."""
    import os

    from helpers import TINY, run_train, write_fake_sbatch

    d = str(tmp_path)
    write_fake_sbatch(d)
    rc, out = run_train(d, "4101", TINY + ["--synthetic-data", "--vocab-size", "256", "--model-dtype", "fp32",
                                           "--training-steps", "3", "--checkpoint-path", os.path.join(d, "ck")])
    assert rc == 0 and "Training completed" in out, out[-2000:]
    assert out.count("--model-dtype fp32: GEMMs on the fp32 MFMA kernel") == 1, out[-2000:]
    rc, out = run_train(d, "4102", TINY + ["--synthetic-data", "--vocab-size", "256", "--training-steps", "2",
                                           "--checkpoint-path", os.path.join(d, "ck")])
    assert rc == 0 and "--model-dtype fp32" not in out


def test_qkv_rope_min_k_knob(monkeypatch):
    """FT_QKV_ROPE_MIN_K (ops/attention.py): the QKV projection with the RoPE epilogue from this model
    dim; 2048 by default (the 8B class), so GPT-2 (768 / 1024) keeps the separate RoPE kernel (the
    fused form measured 0.6-0.7 % slower there: profiles/r6/gpt2_graph_ab.log)."""
    from fault_tolerant_llm_training_amd.ops import attention as A

    a = model_args_for("gpt2-small", vocab_size=50304, seq_len=2048)
    assert routing_table(a, torch.bfloat16)["qkv fwd"] == "w4 128"
    monkeypatch.setattr(A, "_QKV_ROPE_MIN_K", 768)
    assert routing_table(a, torch.bfloat16)["qkv fwd"] == "w4 qkv+rope"
