"""The data-parallel path over RCCL on the GPU (1-rank process group, explicit DP mode).

A single-GPU box cannot host two RCCL ranks (one GPU per rank), so this runs bench.py under
torchrun with one rank and an explicit ``--dp-mode``: the gradient buckets then really go
through RCCL reduce-scatter / all-reduce / all-gather issued from the dW side stream and
the optimizer stream, the sparse embedding exchange all-gathers through RCCL, and the
step must produce the same loss as the local (no collective) run of the same seed.
The multi-rank logic is covered by the gloo tests (test_dp_gloo.py, test_bench_contract.py).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

from helpers import ROOT

pytestmark = pytest.mark.gpu

ARGS = ["--model", "tiny", "--vocab-size", "4096", "--seq-len", "256", "--steps", "3", "--warmup", "1",
        "--bucket-mb", "0.5"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(extra, torchrun):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    if torchrun:
        env["FT_FORCE_DIST"] = "1"  # build the RCCL process group even for one rank
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "1"]
    else:
        cmd = [sys.executable, "bench.py"]
    r = subprocess.run(cmd + ARGS + extra, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return lines[0]


@pytest.mark.parametrize("mode,rdt", [("zero1", "native"), ("allreduce", "native"), ("zero1", "fp32"),
                                      ("allreduce", "fp32")])
def test_rccl_one_rank_matches_local(mode, rdt):
    """fp32: the reduced fp32 copy is written back from the reducer's side stream while its
    buffers were allocated on the launching stream (record_stream keeps them alive)."""
    local = _run([], torchrun=False)
    dp = _run(["--dp-mode", mode, "--dp-reduce-dtype", rdt], torchrun=True)
    assert dp["grad_mode"] == mode and local["grad_mode"] == "local"
    assert dp["world_size"] == 1 and dp["distinct_devices"] == 1
    # same math: the 1-rank collectives are identities; zero1 shards are the whole buckets
    assert abs(dp["final_loss"] - local["final_loss"]) < 1e-3, (dp["final_loss"], local["final_loss"])
