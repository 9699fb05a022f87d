"""Checkpoint engine on the GPU: native HIP snapshot engine (side stream, HBM staging / pinned
D2H), the native O_DIRECT zip writer, fence semantics, and the pinned-ring restore."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", ["hbm", "host"])
def test_snapshot_engine_roundtrip_and_fence(tmp_path, mode):
    from fault_tolerant_llm_training_amd._native import runtime
    from fault_tolerant_llm_training_amd.ckpt.engine import CheckpointEngine
    from fault_tolerant_llm_training_amd.ckpt.format import load_checkpoint

    runtime()  # the native runtime must be present on the GPU box
    n = 3 * (1 << 20) + 64
    bufs = {k: torch.randn(n, device="cuda").bfloat16() for k in ("params", "exp_avg", "exp_avg_sq")}
    ref = {k: v.clone() for k, v in bufs.items()}
    eng = CheckpointEngine(bufs, mode=mode)
    assert eng.mode == mode
    path = str(tmp_path / "g.ckpt")
    st = eng.save(path, lambda h: {"model": {"p": h["params"]}, "m": h["exp_avg"], "v": h["exp_avg_sq"],
                                   "training_step": 3}, blocking=False)
    eng.fence()  # the next "optimizer step" may only run after the snapshot
    for v in bufs.values():
        v.add_(1.0)  # mutate after the fence: must not leak into the file
    st = eng.wait()
    assert st.bytes > 3 * n * 2
    c = load_checkpoint(path)
    assert torch.equal(c["model"]["p"], ref["params"].cpu())
    assert torch.equal(c["m"], ref["exp_avg"].cpu()) and torch.equal(c["v"], ref["exp_avg_sq"].cpu())
    assert c["training_step"] == 3


def test_background_pinned_preallocation(tmp_path):
    """Pinned host buffers allocated by a background thread at startup; "auto" mode is decided
    at the first save, so the early engine reserves no HBM staging copy."""
    from fault_tolerant_llm_training_amd.ckpt.engine import CheckpointEngine
    from fault_tolerant_llm_training_amd.ckpt.format import load_checkpoint

    n = 5 * (1 << 20) + 8
    bufs = {k: torch.randn(n, device="cuda").bfloat16() for k in ("params", "exp_avg", "exp_avg_sq")}
    eng = CheckpointEngine(bufs, mode="auto")
    before = torch.cuda.memory_allocated()
    eng.preallocate_async()
    assert torch.cuda.memory_allocated() == before  # no staging copy yet
    assert eng._mode == "auto"
    path = str(tmp_path / "p.ckpt")
    # the save may race the thread: it blocks on the host-buffer lock, then uses the same buffers
    st = eng.save(path, lambda h: {"m": h["params"], "a": h["exp_avg"], "v": h["exp_avg_sq"]}, blocking=True)
    assert eng.preallocated(30) and eng.prealloc_s is not None
    host_before = {k: v.data_ptr() for k, v in eng.host_views().items()}
    st2 = eng.save(path, lambda h: {"m": h["params"], "a": h["exp_avg"], "v": h["exp_avg_sq"]}, blocking=True)
    assert st2.mode == st.mode
    # the second save reuses the pinned buffers (no new allocation) and the event pool
    assert {k: v.data_ptr() for k, v in eng.host_views().items()} == host_before
    assert eng._eng is None or eng._eng.num_events() <= 3
    assert eng.mode in ("hbm", "host") and st.mode == eng.mode
    assert all(t.is_pinned() for t in eng.host_views().values())
    c = load_checkpoint(path)
    assert torch.equal(c["m"], bufs["params"].cpu()) and torch.equal(c["v"], bufs["exp_avg_sq"].cpu())
