"""GEMM routing table per preset and dtype (ops/routing.py: routing_table evaluates the same
predicates the autograd functions use, on shape/dtype specs: no GPU needed). Pins which kernel
each product of the step takes, so a routing change is a visible test change:

* Llama-3-8B bf16 / fp16: every product on the hand-written w4 kernel -- none on hipBLASLt (the
  deep-reduction dX products with a K split);
* fp32 models and CPU tensors: hipBLASLt / the composed path (the MFMA kernels are 16-bit);
* GPT-2-sized presets at one sequence: the products whose w4 plan fills half the chip on w4,
  the rest (latency-bound) on hipBLASLt.
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
def test_fp32_and_cpu_take_no_mfma_gemm(preset):
    a = model_args_for(preset, vocab_size=50304 if preset != "llama3-8b" else 131072, seq_len=2048)
    assert set(routing_table(a, torch.float32).values()) == {"hipBLASLt"}
    assert set(routing_table(a, torch.bfloat16, cuda=False).values()) == {"hipBLASLt"}


@pytest.mark.parametrize("preset,vocab", [("gpt2-small", 50304), ("gpt2-small", 131072),
                                          ("gpt2-medium", 50304), ("gpt2-medium", 131072)])
def test_gpt2_routes(preset, vocab):
    t = routing_table(model_args_for(preset, vocab_size=vocab, seq_len=2048), torch.bfloat16)
    on_w4 = sorted(k for k, v in t.items() if v.startswith("w4"))
    # the LM-head dX (K = V) always takes a K split on w4; the 768 / 1024-wide projections'
    # forward / dX with enough tiles do too; wo (2048 x D x D, K = D <= 1024) runs its 48-64 tiles
    # on w4 without a split (short reductions, profiles/r5_gpt2_gemm_probe.log), its dW (k-major A,
    # K = 2048 tokens) stays on hipBLASLt
    assert t["head dX"].startswith("w4") and " x" in t["head dX"]
    assert t["wo fwd"] == t["wo dX"] == "w4 128" and t["wo dW"] == "hipBLASLt"
    assert t["qkv fwd"].startswith("w4") and t["w13 dX"].startswith("w4")
    # the head's dW needs V % 256 (rows of the k-major tiles): GPT-2's padded 50304 stays on hipBLASLt
    assert t["head dW"] == ("w4 256" if vocab % 256 == 0 else "hipBLASLt")
    assert len(on_w4) >= 5, t


def test_blas_only_knob(monkeypatch):
    monkeypatch.setattr(Fx, "_BLAS_ONLY", True)
    from fault_tolerant_llm_training_amd.ops import attention as A

    t = routing_table(model_args_for("llama3-8b", vocab_size=131072, seq_len=2048), torch.bfloat16)
    assert set(t.values()) == {"hipBLASLt"}
    assert A._qkv_rope_ok is not None
