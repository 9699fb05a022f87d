"""Sharded multi-writer checkpoint: W gloo ranks each write their pieces of one file."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.slow


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, path, interleaved):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    group = dist.new_group(backend="gloo")
    from fault_tolerant_llm_training_amd.ckpt.engine import CheckpointEngine, Region

    n = 300_001 * 2  # deliberately not a multiple of anything useful
    full = {k: (torch.arange(n, dtype=torch.float32) * (i + 1)).to(torch.bfloat16) for i, k in enumerate(("a", "b"))}
    regions = []
    for k, t in full.items():
        if interleaved:  # ZeRO-1-like: many small pieces per rank, interleaved across ranks
            step = 1000
            pieces, data = [], []
            off = 0
            for j, lo in enumerate(range(0, n, step)):
                if j % world == rank:
                    hi = min(n, lo + step)
                    pieces.append((lo, off, hi - lo))
                    data.append(t[lo:hi])
                    off += hi - lo
            regions.append(Region(k, torch.cat(data) if data else t[:0].clone(), pieces, n))
        else:
            lo, hi = n * rank // world, n * (rank + 1) // world
            regions.append(Region(k, t[lo:hi].clone(), [(lo, 0, hi - lo)], n))
    eng = CheckpointEngine(regions, group=group, rank=rank, world=world)

    def build(host):
        return {"model": {"x": host["a"][10:20], "whole": host["a"]}, "opt": {"b": host["b"]}, "training_step": 7}

    eng.save(path, build, blocking=True)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,interleaved", [(3, False), (2, True), (4, True)])
def test_sharded_save_roundtrip(tmp_path, world, interleaved):
    path = str(tmp_path / "checkpoint_9.ckpt")
    mp.start_processes(_worker, args=(world, _port(), path, interleaved), nprocs=world, start_method="spawn")
    assert not os.path.exists(path + ".tmp")
    c = torch.load(path, map_location="cpu", weights_only=True)
    n = 300_001 * 2
    a = (torch.arange(n, dtype=torch.float32)).to(torch.bfloat16)
    b = (torch.arange(n, dtype=torch.float32) * 2).to(torch.bfloat16)
    assert torch.equal(c["model"]["whole"], a) and torch.equal(c["opt"]["b"], b)
    assert torch.equal(c["model"]["x"], a[10:20]) and c["training_step"] == 7
    import zipfile

    assert zipfile.ZipFile(path).testzip() is None  # combined CRCs are right
