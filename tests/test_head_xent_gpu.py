"""Chunked LM head + cross-entropy (ops/functional.py LMHeadCrossEntropyFn) vs an fp32 reference.

Reference math: logits = h @ W^T (model.py:379), loss = CE(logits.float(), labels, sum,
ignore_index=-100) / num_items (train.py:101-102). The reference here is computed in fp32,
row chunk by row chunk, so T = 65536 x V = 131072 fits; it checks loss, dh and dW.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(h, w, lab, inv, rows=4096):
    hf, wf = h.float(), w.float()
    loss = torch.zeros((), dtype=torch.float64, device=h.device)
    dh = torch.empty_like(hf)
    dw = torch.zeros_like(wf)
    for r0 in range(0, h.shape[0], rows):
        hc = hf[r0:r0 + rows].requires_grad_(True)
        wc = wf.detach().requires_grad_(True)
        lg = hc @ wc.t()
        l = torch.nn.functional.cross_entropy(lg, lab[r0:r0 + rows], reduction="sum", ignore_index=-100) * inv
        a, b = torch.autograd.grad(l, (hc, wc))
        loss += l.double()
        dh[r0:r0 + rows] = a
        dw += b
    return loss.float(), dh, dw


def _rel(a, b):
    return ((a.float() - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("T,V,D,chunk_mb", [(2048, 131072, 256, 256.0), (65536, 131072, 128, 256.0),
                                            (1024, 8192, 512, 1.0), (512, 4096, 256, 1024.0)])
def test_chunked_head_xent_matches_fp32(T, V, D, chunk_mb, monkeypatch):
    from fault_tolerant_llm_training_amd.ops import functional as Fx

    monkeypatch.setattr(Fx, "_HEAD_CHUNK_MB", chunk_mb)
    torch.manual_seed(T + V)
    h = (torch.randn(T, D, device="cuda") * 2).bfloat16().requires_grad_(True)
    w = (torch.randn(V, D, device="cuda") * 0.05).bfloat16().requires_grad_(True)
    lab = torch.randint(0, V, (T,), device="cuda")
    lab[::7] = -100  # ignore_index rows
    n = (lab != -100).sum()
    inv = (1.0 / n.float()).reshape(1)
    rows = Fx._head_rows(T, V)
    if chunk_mb <= 256 and V == 131072:
        assert rows * V * 2 <= 256 * 2**20 and rows < T  # never the whole [T, V] logits
    loss = Fx.lm_head_cross_entropy(h, w, lab, inv)
    loss.backward()
    rl, rdh, rdw = _ref(h.detach(), w.detach(), lab, inv.item())
    assert abs(loss.item() - rl.item()) <= 2e-3 * abs(rl.item()) + 1e-3, (loss.item(), rl.item())
    assert _rel(h.grad, rdh) < 2e-2
    assert _rel(w.grad, rdw) < 2e-2
    assert torch.isfinite(h.grad.float()).all()


def test_chunked_head_upstream_grad_and_accumulate():
    """g != 1 is applied in backward; a sink in accumulate mode takes the recompute path."""
    from fault_tolerant_llm_training_amd.ops import functional as Fx
    from fault_tolerant_llm_training_amd.ops.grad_sink import GradSink

    T, V, D = 1024, 8192, 256
    h = torch.randn(T, D, device="cuda").bfloat16().requires_grad_(True)
    w = (torch.randn(V, D, device="cuda") * 0.05).bfloat16()
    lab = torch.randint(0, V, (T,), device="cuda")
    inv = torch.full((1,), 1.0 / T, device="cuda")
    buf = torch.zeros(V * D, dtype=torch.bfloat16, device="cuda")
    sink = GradSink(buf, 0, V * D)
    (Fx.lm_head_cross_entropy(h, w, lab, inv, sink) * 3.0).backward()
    g1 = buf.clone().float()
    dh1 = h.grad.clone().float()
    _, rdh, rdw = _ref(h.detach(), w, lab, 1.0 / T)
    assert _rel(dh1, 3 * rdh) < 2e-2 and _rel(g1.view(V, D), 3 * rdw) < 2e-2
    h.grad = None
    sink.accumulate = True  # second micro-batch adds on top
    Fx.lm_head_cross_entropy(h, w, lab, inv, sink).backward()
    assert _rel(buf.float().view(V, D), 4 * rdw) < 2e-2
