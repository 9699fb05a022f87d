"""Process-group bootstrap: one process per GPU, RCCL data plane + gloo control plane.

The reference is single-process (train.sh:5-7; LOCAL_RANK only picks the
device, train.py:16). Here ranks come from torchrun (RANK/LOCAL_RANK/WORLD_SIZE)
or Slurm (SLURM_PROCID/SLURM_LOCALID/SLURM_NTASKS). Two groups are created:

* the default group on ``nccl`` (= RCCL on ROCm, over xGMI inside a node) for
  gradient all-reduce — stream-ordered, never blocks the host;
* a ``gloo`` CPU group for control-plane agreement (stop-signal consensus,
  token counts, data-loader states, config checks), so a 4-byte vote never
  forces a GPU synchronisation;
* a second ``gloo`` group with a SHORT timeout (``--peer-timeout``, default
  60 s) used only by the per-step vote: a peer that died (SIGKILL, OOM kill)
  closes its sockets and fails the vote at once; one that hangs fails it after
  the timeout. Either way the survivors learn it well inside Slurm's 120 s
  ``USR1`` lead instead of the 30-minute default collective timeout, and
  :class:`PeerFailure` is raised.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    ctrl_group: Optional[object] = None  # gloo group (None when world_size == 1)
    ckpt_group: Optional[object] = None  # gloo group used only by checkpoint writer threads
    vote_group: Optional[object] = None  # gloo group with the short peer timeout (per-step vote)
    peer_timeout_s: float = 60.0

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1 or self.ctrl_group is not None


_INFO: Optional[DistInfo] = None


class PeerFailure(RuntimeError):
    """A peer rank stopped answering the control plane (died, or hung past the peer timeout)."""


def env_ranks():
    env = os.environ
    if "RANK" in env and "WORLD_SIZE" in env:
        return int(env["RANK"]), int(env["WORLD_SIZE"]), int(env.get("LOCAL_RANK", 0))
    if "SLURM_PROCID" in env and "SLURM_NTASKS" in env:
        return int(env["SLURM_PROCID"]), int(env["SLURM_NTASKS"]), int(env.get("SLURM_LOCALID", 0))
    return 0, 1, int(env.get("LOCAL_RANK", 0))


def init_distributed(device_type: str = "cuda", timeout_s: int = 1800, peer_timeout_s: float = 60.0) -> DistInfo:
    global _INFO
    if _INFO is not None:
        return _INFO
    rank, world, local = env_ranks()
    if device_type == "cuda":
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    info = DistInfo(rank, world, local, device, peer_timeout_s=float(peer_timeout_s))
    # FT_FORCE_DIST=1 builds the process groups even for one rank (exercises the RCCL path on 1 GPU)
    if world > 1 or os.environ.get("FT_FORCE_DIST") == "1":
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        os.environ["RANK"], os.environ["WORLD_SIZE"] = str(rank), str(world)
        timeout = datetime.timedelta(seconds=timeout_s)
        # RCCL kernels on a high-priority stream: the bucket collectives that overlap
        # backward / the next forward get CU slots ahead of queued GEMM workgroups
        os.environ.setdefault("TORCH_NCCL_HIGH_PRIORITY", "1")
        if not dist.is_initialized():
            if device_type == "cuda":
                dist.init_process_group("nccl", timeout=timeout, device_id=device)
            else:
                dist.init_process_group("gloo", timeout=timeout)
        info.ctrl_group = dist.new_group(backend="gloo", timeout=timeout) if device_type == "cuda" else dist.group.WORLD
        # a second gloo group so background checkpoint-writer threads never interleave
        # their collectives with the main thread's control-plane votes
        info.ckpt_group = dist.new_group(backend="gloo", timeout=timeout)
        info.vote_group = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=peer_timeout_s))
    _INFO = info
    return info


def get_info() -> DistInfo:
    return _INFO if _INFO is not None else DistInfo()


def ctrl_allreduce_max(value: int) -> int:
    """Host-side MAX vote over the gloo control group (no GPU sync)."""
    info = get_info()
    if not info.distributed:
        return value
    t = torch.tensor([value], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=info.ctrl_group)
    return int(t.item())


def ctrl_allreduce_sum(value: float) -> float:
    info = get_info()
    if not info.distributed:
        return value
    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=info.ctrl_group)
    return float(t.item())


def ctrl_all_gather_object(obj):
    info = get_info()
    if not info.distributed:
        return [obj]
    out = [None] * info.world_size
    dist.all_gather_object(out, obj, group=info.ctrl_group)
    return out


def ctrl_broadcast_object(obj, src: int = 0):
    info = get_info()
    if not info.distributed:
        return obj
    box = [obj]
    dist.broadcast_object_list(box, src=src, group=info.ctrl_group)
    return box[0]


def vote(values):
    """All-gather a short float vector from every rank over the short-timeout gloo group.

    Returns a [world, len(values)] float64 tensor (row r = rank r's values); every rank
    gets the same table, so MAX/SUM/first-rank decisions taken from it agree. Any
    failure of the exchange (peer gone or hung past ``--peer-timeout``) raises
    :class:`PeerFailure`."""
    info = get_info()
    t = torch.tensor([float(v) for v in values], dtype=torch.float64)
    if not info.distributed:
        return t.view(1, -1)
    out = torch.empty(info.world_size * t.numel(), dtype=torch.float64)
    try:
        dist.all_gather_into_tensor(out, t, group=info.vote_group)
    except Exception as e:  # noqa: BLE001 - gloo raises RuntimeError/DistBackendError subclasses
        raise PeerFailure(f"step vote failed (peer rank lost or hung > {info.peer_timeout_s:.0f}s): {e}") from e
    return out.view(info.world_size, -1)


def barrier():
    info = get_info()
    if info.distributed:
        dist.barrier(group=info.ctrl_group)


def destroy():
    global _INFO
    if dist.is_initialized():
        dist.destroy_process_group()
    _INFO = None
