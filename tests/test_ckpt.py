"""Checkpoint format, native writer, engine, restore paths (reference utils.py:74-81, train.py:20-84)."""
import os
import zipfile

import pytest
import torch

from fault_tolerant_llm_training_amd._native import runtime_available
from fault_tolerant_llm_training_amd.ckpt.engine import CheckpointEngine
from fault_tolerant_llm_training_amd.ckpt.format import checkpoint_file, load_checkpoint
from fault_tolerant_llm_training_amd.ckpt.state import build_checkpoint, restore_model
from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for
from fault_tolerant_llm_training_amd.optim.adamw import FlatAdamW
from fault_tolerant_llm_training_amd.utils.lr import build_lr_scheduler


def _setup(seed=0, dtype=torch.bfloat16):
    a = model_args_for("tiny", vocab_size=96, seq_len=16)
    m = build_model(a, "cpu", dtype, seed=seed)
    opt = FlatAdamW(m.parameters(), m.flat, lr=1e-3, max_grad_norm=1.0)
    s = build_lr_scheduler(opt, 3)
    tok = torch.randint(0, 96, (2, 16))
    m(tok, tok).backward()
    opt.step()
    s.step()
    return m, opt, s


def _engine(m, opt):
    return CheckpointEngine({"params": m.flat.params, "exp_avg": opt.exp_avg, "exp_avg_sq": opt.exp_avg_sq})


def test_checkpoint_path_contract():
    assert checkpoint_file("/x/checkpoints", 444664) == "/x/checkpoints/checkpoint_444664.ckpt"


@pytest.mark.parametrize("native", [True, False])
def test_save_load_roundtrip_reference_keys(tmp_path, native, monkeypatch):
    if native and not runtime_available():
        pytest.skip("native runtime not built")
    m, opt, s = _setup()
    eng = _engine(m, opt)
    eng.native = native
    path = checkpoint_file(str(tmp_path / "ck"), 7)
    st = eng.save(path, lambda host: build_checkpoint(m, opt, s, 5, host, data_loader={"kind": "x", "next_step": 5}),
                  step=5, blocking=True)
    assert st.total_s > 0 and os.path.exists(path) and not os.path.exists(path + ".tmp")
    c = torch.load(path, map_location="cpu", weights_only=True)  # what the reference loader does
    assert set(c) >= {"model", "optimizer", "lr_scheduler", "training_step"}
    assert c["training_step"] == 5
    assert list(c["model"].keys()) == list(m.state_dict().keys())
    for k, v in m.state_dict().items():
        assert torch.equal(c["model"][k], v), k
    ref_sd = opt.state_dict()
    assert c["optimizer"]["param_groups"][0]["lr"] == ref_sd["param_groups"][0]["lr"]
    for i, e in ref_sd["state"].items():
        assert torch.equal(c["optimizer"]["state"][i]["exp_avg"], e["exp_avg"])
        assert float(c["optimizer"]["state"][i]["step"]) == 1.0
    assert c["lr_scheduler"]["last_epoch"] == s.last_epoch
    if native:
        # one storage per flat buffer (+ the small step tensors)
        z = zipfile.ZipFile(path)
        big = [i for i in z.infolist() if "/data/" in i.filename and i.file_size > 1000]
        assert len(big) == 3
        assert z.testzip() is None  # CRCs are right


def test_restore_fast_and_per_tensor_paths(tmp_path):
    m, opt, s = _setup(seed=1)
    eng = _engine(m, opt)
    path = str(tmp_path / "a.ckpt")
    eng.save(path, lambda host: build_checkpoint(m, opt, s, 3, host), blocking=True)
    c = load_checkpoint(path)
    m2, opt2, s2 = _setup(seed=2)
    assert restore_model(m2, c["model"]) == "flat"
    assert torch.equal(m2.flat.params, m.flat.params)
    opt2.load_state_dict(c["optimizer"])
    assert torch.equal(opt2.exp_avg, opt.exp_avg) and torch.equal(opt2.exp_avg_sq, opt.exp_avg_sq)
    assert opt2.step_count == opt.step_count
    # a reference-style file: plain torch.save of per-tensor clones, with torch.compile's prefix
    ref = {"model": {"_orig_mod." + k: v.clone() for k, v in m.state_dict().items()},
           "optimizer": opt.state_dict(), "lr_scheduler": s.state_dict(), "training_step": 3}
    for e in ref["optimizer"]["state"].values():
        e["exp_avg"], e["exp_avg_sq"] = e["exp_avg"].clone(), e["exp_avg_sq"].clone()
    torch.save(ref, str(tmp_path / "ref.ckpt"))
    c2 = load_checkpoint(str(tmp_path / "ref.ckpt"))
    m3, opt3, _ = _setup(seed=3)
    assert restore_model(m3, c2["model"]) == "per-tensor"
    assert torch.equal(m3.flat.params, m.flat.params)
    opt3.load_state_dict(c2["optimizer"])
    assert torch.equal(opt3.exp_avg, opt.exp_avg)


def test_strict_load_rejects_mismatch():
    m, _, _ = _setup()
    sd = dict(m.state_dict())
    sd.pop("norm.weight")
    with pytest.raises(KeyError):
        restore_model(m, sd)


def test_our_file_loads_into_plain_torch_adamw(tmp_path):
    """Interop: the optimizer entry has torch AdamW's structure."""
    m, opt, s = _setup()
    path = str(tmp_path / "b.ckpt")
    _engine(m, opt).save(path, lambda host: build_checkpoint(m, opt, s, 1, host), blocking=True)
    c = torch.load(path, map_location="cpu", weights_only=True)
    params = [torch.nn.Parameter(v.clone().float()) for v in m.state_dict().values()]
    t_opt = torch.optim.AdamW(params, lr=1e-3)
    t_opt.load_state_dict(c["optimizer"])
    for p in params:
        p.grad = torch.zeros_like(p)
    t_opt.step()


def test_async_save_overlaps_and_snapshot_is_consistent(tmp_path):
    m, opt, s = _setup()
    eng = _engine(m, opt)
    before = m.flat.params.clone()
    path = str(tmp_path / "c.ckpt")
    eng.save(path, lambda host: build_checkpoint(m, opt, s, 1, host), blocking=False)
    m.flat.params.add_(1.0)  # training continues and mutates the live buffer
    st = eng.wait()
    assert st is not None and st.path == path
    c = load_checkpoint(path)
    assert restore_model(m, c["model"]) == "flat"
    assert torch.equal(m.flat.params, before)


def test_failed_publish_raises_and_leaves_no_partial_file(tmp_path):
    m, opt, s = _setup()
    eng = _engine(m, opt)
    target = tmp_path / "e.ckpt"
    os.makedirs(target / "occupied")  # rename(tmp -> non-empty dir) must fail
    with pytest.raises(RuntimeError):
        eng.save(str(target), lambda host: build_checkpoint(m, opt, s, 2, host), blocking=True)
    assert os.path.isdir(target)
    # the engine is usable again afterwards
    ok = str(tmp_path / "f.ckpt")
    eng.save(ok, lambda host: build_checkpoint(m, opt, s, 2, host), blocking=True)
    assert load_checkpoint(ok)["training_step"] == 2


def test_file_reader_ranges(tmp_path):
    """Native parallel pread (O_DIRECT bodies + buffered head/tail) returns the file's bytes."""
    from fault_tolerant_llm_training_amd._native import runtime

    data = torch.randint(0, 256, (3 * (1 << 20) + 12345,), dtype=torch.uint8)
    p = tmp_path / "blob.bin"
    p.write_bytes(data.numpy().tobytes())
    r = runtime().FileReader(str(p), 4, True)
    for off, n in ((0, data.numel()), (4096, 1 << 20), (8192, 12345), (77, 5000), (1 << 20, 2 * (1 << 20) + 12345)):
        out = torch.empty(n, dtype=torch.uint8)
        r.read(off, out.data_ptr(), n)
        assert torch.equal(out, data[off : off + n]), (off, n)
    assert r.bytes > 0
    with pytest.raises(RuntimeError):
        out = torch.empty(100, dtype=torch.uint8)
        r.read(data.numel() - 10, out.data_ptr(), 100)  # past the end of the file


def test_file_backing_of_mmap_checkpoint(tmp_path):
    """A tensor of torch.load(mmap=True) maps the checkpoint file; the reported offset holds its bytes."""
    from fault_tolerant_llm_training_amd.ckpt.restore import file_backing

    t = torch.randn(1 << 18)
    p = tmp_path / "ck.pt"
    torch.save({"a": torch.arange(10), "t": t}, str(p))
    sd = torch.load(str(p), mmap=True, weights_only=True)
    fb = file_backing(sd["t"])
    assert fb is not None and os.path.samefile(fb[0], str(p))
    with open(p, "rb") as f:
        f.seek(fb[1])
        raw = f.read(t.numel() * 4)
    assert torch.equal(torch.frombuffer(bytearray(raw), dtype=torch.float32), t)
    assert file_backing(torch.randn(100)) is None


def test_background_preallocation_cpu(tmp_path):
    m, opt, s = _setup()
    eng = _engine(m, opt)
    eng.preallocate_async()
    assert eng.preallocated(30)
    host = eng.host_views()
    path = checkpoint_file(str(tmp_path / "ck"), 9)
    eng.save(path, lambda h: build_checkpoint(m, opt, s, 2, h), step=2, blocking=True)
    assert eng.host_views() is host  # the save reused the preallocated buffers
    c = torch.load(path, map_location="cpu", weights_only=True)
    for k, v in m.state_dict().items():
        assert torch.equal(c["model"][k], v), k


@pytest.mark.parametrize("src,dst", [(torch.float16, torch.float32), (torch.float32, torch.float16)])
def test_moment_dtype_converts_on_load(tmp_path, src, dst):
    """fp16 models keep fp32 AdamW moments by default (the reference keeps them in the model dtype,
    docs/PARITY.md): a checkpoint written with the other moment dtype — an fp16-moment file from an
    earlier / reference-style run, or the reverse — loads with the values converted, both through
    the flat fast path and the per-tensor path."""
    a = model_args_for("tiny", vocab_size=96, seq_len=16)
    m = build_model(a, "cpu", torch.float16, seed=4)
    opt = FlatAdamW(m.parameters(), m.flat, lr=1e-3, max_grad_norm=1.0, state_dtype=src)
    tok = torch.randint(0, 96, (2, 16))
    m(tok, tok).backward()
    opt.step()
    path = str(tmp_path / "m.ckpt")
    s = build_lr_scheduler(opt, 3)
    _engine(m, opt).save(path, lambda host: build_checkpoint(m, opt, s, 1, host), blocking=True)
    c = load_checkpoint(path)
    assert c["optimizer"]["state"][0]["exp_avg"].dtype == src
    m2 = build_model(a, "cpu", torch.float16, seed=5)
    opt2 = FlatAdamW(m2.parameters(), m2.flat, lr=1e-3, max_grad_norm=1.0, state_dtype=dst)
    opt2.load_state_dict(c["optimizer"])
    assert opt2.exp_avg.dtype == dst
    assert torch.equal(opt2.exp_avg, opt.exp_avg.to(dst)) and torch.equal(opt2.exp_avg_sq, opt.exp_avg_sq.to(dst))
    assert opt2.step_count == opt.step_count
