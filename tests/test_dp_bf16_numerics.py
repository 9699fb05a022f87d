"""bf16 data-parallel gradient numerics at W = 8 (gloo on the CPU; RCCL reduces bf16 the same way:
each hop adds in fp32 and rounds back to bf16).

The DP gradient of the tiny model (bf16 parameters, bf16 gradient buckets reduced as bf16 SUM,
reduce-scatter under ZeRO-1 or all-reduce) is compared with the single-process **fp32**
gradient of the same global batch. Two numbers per run:

* ``dp``  = ||g_dp - g_fp32|| / ||g_fp32||     (bf16 compute + bf16 reduction)
* ``one`` = ||g_1 - g_fp32|| / ||g_fp32||      (bf16 compute of the global batch in ONE process)

The documented bound (docs/PERFORMANCE.md, "DP gradient numerics"): ``dp <= one + 2^-8`` —
the bf16 reduction over 8 ranks adds less than one bf16 unit roundoff (2^-8) of relative error
on top of what bf16 compute alone costs (measured: +1.1e-3 = 0.29 * 2^-8, 6.2e-3 vs 5.1e-3), and
every parameter tensor stays within ``4 * 2^-8`` of fp32 in relative L2 (measured 2.3 * 2^-8).
``--dp-reduce-dtype fp32`` (opt-in) reduces an fp32 copy of each bucket instead and lands within
``0.25 * 2^-8`` of the one-process bf16 gradient (measured +0.24e-3).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.slow

WORLD = 8
U = 2.0 ** -8  # bf16 unit roundoff


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(world):
    from fault_tolerant_llm_training_amd.data.synthetic import SyntheticTokens

    xs, ys = [], []
    for r in range(world):
        x, y = SyntheticTokens(128, 32, seed=9, rank=r, world_size=world, pin=False).batch(0, 2)
        y[0, :3] = -100
        xs.append(x)
        ys.append(y)
    return xs, ys


def _worker(rank, world, port, out_dir, mode, reduce_dtype):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for
    from fault_tolerant_llm_training_amd.parallel.ddp import GradReducer

    a = model_args_for("tiny", vocab_size=128, seq_len=32)
    m = build_model(a, "cpu", torch.bfloat16, seed=5)
    ddp = GradReducer(m.flat, m.sinks_in_backward_order(), bucket_mb=0.05, mode=mode, reduce_dtype=reduce_dtype)
    xs, ys = _batch(world)
    x, y = xs[rank], ys[rank]
    n = float(sum(int((t != -100).sum()) for t in ys))
    loss = m(x, y, torch.tensor([1.0 / n]))
    loss.backward()
    ddp.finish()
    full = torch.full(m.flat.grads.shape, float("nan"), dtype=torch.float32)
    for b in ddp.buckets:
        if mode == "zero1" and not b.sparse:
            lo = b.lo + rank * b.shard_len
            full[lo : lo + b.shard_len] = ddp.grad_for_update(b).float()
        elif mode == "zero1":
            lo = b.lo + rank * b.shard_len
            full[lo : lo + b.shard_len] = m.flat.grads[lo : lo + b.shard_len].float()
        else:
            full[b.lo : b.hi] = m.flat.grads[b.lo : b.hi].float()
    torch.save(full, os.path.join(out_dir, f"g{rank}.pt"))
    dist.destroy_process_group()


def _single(dtype):
    from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for

    a = model_args_for("tiny", vocab_size=128, seq_len=32)
    m = build_model(a, "cpu", torch.bfloat16, seed=5)  # the same bf16 weights
    if dtype != torch.bfloat16:
        m32 = build_model(a, "cpu", dtype, seed=5)
        m32.flat.params.copy_(m.flat.params.to(dtype))
        m = m32
    xs, ys = _batch(WORLD)
    loss = m(torch.cat(xs), torch.cat(ys))
    loss.backward()
    return m, m.flat.grads.float().clone()


def _rel(a, b):
    return float((a - b).norm() / b.norm())


@pytest.mark.parametrize("mode,reduce_dtype", [("zero1", "bf16"), ("allreduce", "bf16"), ("zero1", "fp32")])
def test_bf16_dp8_gradient_within_documented_bound(tmp_path, mode, reduce_dtype):
    mp.start_processes(_worker, args=(WORLD, _free_port(), str(tmp_path), mode, reduce_dtype), nprocs=WORLD,
                       start_method="spawn")
    gs = [torch.load(tmp_path / f"g{r}.pt") for r in range(WORLD)]
    g = gs[0]
    for o in gs[1:]:
        if mode == "allreduce":
            assert torch.equal(o, gs[0])  # replicated: every rank holds the same reduced gradient
        g = torch.where(torch.isnan(g), o, g)
    assert not torch.isnan(g).any()
    m32, g32 = _single(torch.float32)
    _m1, g1 = _single(torch.bfloat16)
    dp, one = _rel(g, g32), _rel(g1, g32)
    print(f"\n[{mode}/{reduce_dtype}] rel L2 vs fp32: dp8 {dp:.3e}  one-process bf16 {one:.3e}")
    assert dp <= one + U, (dp, one)
    if reduce_dtype == "fp32":
        assert dp <= one + 0.25 * U, (dp, one)
    worst = 0.0
    for name, slot in m32.flat.slots.items():
        sl = slice(slot.offset, slot.offset + slot.numel)
        ref = g32[sl]
        if ref.norm() > 0:
            worst = max(worst, _rel(g[sl], ref))
    print(f"[{mode}/{reduce_dtype}] worst per-tensor rel L2: {worst:.3e}")
    assert worst <= 4 * U, worst
