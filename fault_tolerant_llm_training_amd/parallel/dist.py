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


def graph_capture_env() -> None:
    """Before the process group exists, for runs that capture RCCL collectives into a HIP graph.

    The whole-step graph issues its collectives blocking on one stream (ddp.GradReducer
    .single_stream). ProcessGroupNCCL hands the watchdog thread the works of those collectives,
    captured ones included, and the watchdog's hipEventQuery on an event recorded during capture
    fails with hipErrorCapturedEvent. By default the watchdog rethrows that and aborts the process
    (SIGABRT, seen as a race on the 1-rank RCCL tests). With TORCH_NCCL_RETHROW_CUDA_ERRORS=0 it
    logs the error and stops. The job loses only the watchdog's collective timeout, which this
    framework does not rely on: a lost or hung peer is detected by the per-step gloo vote
    (--peer-timeout) and the bounded device drain in the trainer."""
    os.environ.setdefault("TORCH_NCCL_RETHROW_CUDA_ERRORS", "0")


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


def _device_id(device: torch.device) -> dict:
    """Identity of the GPU this rank drives (CPU ranks: host name + rank)."""
    if device.type != "cuda":
        import socket

        return {"type": "cpu", "id": f"{socket.gethostname()}:cpu"}
    p = torch.cuda.get_device_properties(device)
    uuid = getattr(p, "uuid", None)
    bus = getattr(p, "pci_bus_id", None)
    dom = getattr(p, "pci_domain_id", None)
    return {"type": "cuda", "index": device.index, "name": p.name,
            "pci": f"{dom or 0:04x}:{bus:02x}" if bus is not None else None,
            "id": str(uuid) if uuid is not None else f"pci:{dom}:{bus}:{device.index}"}


def topology_report(info: DistInfo, expected_world: Optional[int] = None) -> dict:
    """What the job actually ran on, gathered over the control plane (every rank calls this).

    ``world_size`` from the process group, every rank's device identity, the number of distinct
    GPUs, xGMI/PCIe peer access between every pair of the job's local devices and the RCCL
    version. Raises if a CUDA job runs fewer distinct GPUs than ranks (two ranks sharing one
    GPU would time-slice it and make a scaling number meaningless) or if the process group's
    size differs from ``expected_world``."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    devs = ctrl_all_gather_object(_device_id(info.device))
    ids = [d["id"] for d in devs]
    rep = {"world_size": world, "devices": devs, "distinct_devices": len(set(ids))}
    if info.device.type == "cuda":
        local = sorted({d["index"] for d in devs})
        peer = True
        for i in local:
            for j in local:
                if i != j and not torch.cuda.can_device_access_peer(i, j):
                    peer = False
        rep["peer_access_all_pairs"] = peer if len(local) > 1 else None
        try:
            v = torch.cuda.nccl.version()
            rep["rccl_version"] = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
        except Exception:  # noqa: BLE001 - informational
            rep["rccl_version"] = None
        if rep["distinct_devices"] < world:
            raise RuntimeError(f"{world} ranks but only {rep['distinct_devices']} distinct GPUs: {ids}")
    else:
        rep["peer_access_all_pairs"] = None
        rep["rccl_version"] = None
    if expected_world is not None and world != expected_world:
        raise RuntimeError(f"process group has {world} ranks, expected {expected_world}")
    return rep


def barrier():
    info = get_info()
    if info.distributed:
        dist.barrier(group=info.ctrl_group)


def destroy():
    global _INFO
    if dist.is_initialized():
        dist.destroy_process_group()
    _INFO = None
