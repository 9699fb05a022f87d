#!/usr/bin/env python3
"""Which RCCL collective pattern of the ZeRO-1 step breaks under HIP-graph stream capture?

Each case runs in its own child process (a segfault ends only that child) on a 1-rank RCCL process
group, with faulthandler on so a crash prints the Python frame it happened in. The cases mirror
the calls the ZeRO-1 step makes (parallel/ddp.py, optim/adamw.py): the in-place bucket
reduce-scatter waited for on a side stream, the blocking 4-byte norm all-reduce on that stream,
the in-place parameter all-gather whose work object the next forward waits on (ParamGate).

    python scripts/capture_collectives_probe.py            # every case, one child each
    python scripts/capture_collectives_probe.py --case NAME
    python scripts/capture_collectives_probe.py --only a,b --env K=V

Finding (ROCm 7 / RCCL 2.26 / torch 2.10, profiles/r6/capture_collectives_probe.log): every single
collective captures; RCCL collectives captured on MORE THAN ONE stream in one graph -- an async one
(ProcessGroupNCCL's internal stream) next to a blocking one on ours, or blocking ones on two of our
streams -- crash hipStreamEndCapture with SIGSEGV (zero1_sequence, rs_then_ag_side, comm_stream_*);
any number of them issued blocking on ONE stream, with compute-stream round trips in between, capture
and replay correctly (side_*, all_sync_side). Keeping the works alive, TORCH_NCCL_AVOID_RECORD_STREAMS,
TORCH_NCCL_CUDA_EVENT_CACHE=0 or an anchor kernel before each collective change nothing. The fix:
ddp.GradReducer.single_stream (set by graphs.GraphedStep).
"""
from __future__ import annotations

import argparse
import faulthandler
import os
import socket
import subprocess
import sys

CASES = ["allreduce_async", "allreduce_sync_side", "reduce_scatter_inplace", "reduce_scatter_outofplace",
         "allgather_inplace", "allgather_outofplace", "allgather_inplace_wait_other_stream",
         "zero1_sequence", "rs_then_ar_side", "ar_then_ag_side", "rs_then_ag_side", "two_async_side",
         "zero1_gate_wait_on_side", "zero1_async_norm", "ar_clone_side", "zero1_no_clone",
         "rs_then_ag_keep", "two_async_keep", "zero1_keep",
         "all_sync_side", "rs_oop_then_ag_side", "rs_then_ag_oop", "rs_side_then_ag_side",
         "comm_stream_zero1", "comm_stream_zero1_lowprio", "comm_stream_rs_ag", "comm_stream_rs_ar",
         "comm_stream_zero1_anchor", "comm_stream_rs_ag_anchor",
         "side_zero1", "side_rs_mul_ag", "side_rs_ag", "side_two_buckets", "side_ar_mul_ag", "side_rs_ar_ag_sync",
         "side_roundtrip", "side_roundtrip_rs_first"]
KEEP = []  # *_keep cases: every work object of the capture stays referenced until after capture_end


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def child(case: str) -> None:
    faulthandler.enable(all_threads=True)
    import torch
    import torch.distributed as dist

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    n = 1 << 16
    buf = torch.arange(n, device=dev, dtype=torch.float32)
    other = torch.zeros(n, device=dev, dtype=torch.float32)
    side = torch.cuda.Stream(device=dev)
    comm = torch.cuda.Stream(device=dev, priority=0 if case.endswith("lowprio") else -1)
    evs = [torch.cuda.Event() for _ in range(4)]
    tot1 = torch.zeros(1, device=dev)
    anchor = torch.zeros(1, device=dev)
    cur = torch.cuda.current_stream()

    def body():
        if case == "allreduce_async":
            w = dist.all_reduce(buf, async_op=True)
            w.wait()
        elif case == "allreduce_sync_side":
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                dist.all_reduce(buf[:1])
            torch.cuda.current_stream().wait_stream(side)
        elif case == "reduce_scatter_inplace":
            w = dist.reduce_scatter_tensor(buf, buf, async_op=True)  # 1 rank: own chunk == whole
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                w.wait()
            torch.cuda.current_stream().wait_stream(side)
        elif case == "reduce_scatter_outofplace":
            w = dist.reduce_scatter_tensor(other, buf, async_op=True)
            w.wait()
        elif case == "allgather_inplace":
            w = dist.all_gather_into_tensor(buf, buf, async_op=True)
            w.wait()
        elif case == "allgather_outofplace":
            w = dist.all_gather_into_tensor(other, buf, async_op=True)
            w.wait()
        elif case == "allgather_inplace_wait_other_stream":
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                w = dist.all_gather_into_tensor(buf, buf, async_op=True)
            w.wait()  # on the capture's origin stream (ParamGate.wait in the next forward)
        elif case == "zero1_sequence":
            # backward: bucket reduce-scatter from the compute stream, waited for on the side stream
            w = dist.reduce_scatter_tensor(buf, buf, async_op=True)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                w.wait()
                tot = buf[:1].clone()
                dist.all_reduce(tot)  # global_sumsq (blocking form)
                buf.mul_(1.0)
                g = dist.all_gather_into_tensor(buf, buf, async_op=True)  # parameter all-gather
            g.wait()  # next forward's gate
            torch.cuda.current_stream().wait_stream(side)
        elif case == "rs_then_ar_side":
            w = dist.reduce_scatter_tensor(buf, buf, async_op=True)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                w.wait()
                dist.all_reduce(buf[:1])
            torch.cuda.current_stream().wait_stream(side)
        elif case == "ar_then_ag_side":
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                dist.all_reduce(buf[:1])
                g = dist.all_gather_into_tensor(buf, buf, async_op=True)
            g.wait()
            torch.cuda.current_stream().wait_stream(side)
        elif case in ("rs_then_ag_keep", "two_async_keep", "zero1_keep"):
            if case == "two_async_keep":
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    a1 = dist.all_reduce(buf[:1], async_op=True)
                    a2 = dist.all_gather_into_tensor(buf, buf, async_op=True)
                    a1.wait()
                a2.wait()
                KEEP.extend([a1, a2])
            else:
                w = dist.reduce_scatter_tensor(buf, buf, async_op=True)
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    w.wait()
                    if case == "zero1_keep":
                        tot = buf[:1].clone()
                        dist.all_reduce(tot)
                        buf.mul_(1.0)
                    g = dist.all_gather_into_tensor(buf, buf, async_op=True)
                g.wait()
                KEEP.extend([w, g])
            torch.cuda.current_stream().wait_stream(side)
        elif case == "all_sync_side":
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                dist.reduce_scatter_tensor(buf, buf)
                dist.all_reduce(other[:1])
                dist.all_gather_into_tensor(buf, buf)
            torch.cuda.current_stream().wait_stream(side)
        elif case == "rs_oop_then_ag_side":
            w = dist.reduce_scatter_tensor(other, buf, async_op=True)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                w.wait()
                g = dist.all_gather_into_tensor(buf, buf, async_op=True)
            g.wait()
            torch.cuda.current_stream().wait_stream(side)
        elif case == "rs_then_ag_oop":
            w = dist.reduce_scatter_tensor(buf, buf, async_op=True)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                w.wait()
                g = dist.all_gather_into_tensor(other, buf, async_op=True)
            g.wait()
            torch.cuda.current_stream().wait_stream(side)
        elif case == "rs_side_then_ag_side":
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                w = dist.reduce_scatter_tensor(buf, buf, async_op=True)
                w.wait()
                g = dist.all_gather_into_tensor(buf, buf, async_op=True)
            g.wait()
            torch.cuda.current_stream().wait_stream(side)
        elif case.startswith("side_roundtrip"):
            # the captured ZeRO-1 step: [optimizer(k): norm all-reduce, AdamW, all-gather] on the side
            # stream, the next forward (compute) waits for the all-gather, the next backward's
            # reduce-scatter (side) waits for the compute stream again
            evs[0].record()
            side.wait_event(evs[0])
            with torch.cuda.stream(side):
                if case == "side_roundtrip_rs_first":
                    dist.reduce_scatter_tensor(buf, buf)
                dist.all_reduce(tot1)
                buf.mul_(1.0)
                dist.all_gather_into_tensor(buf, buf)
                evs[1].record()
            torch.cuda.current_stream().wait_event(evs[1])
            buf.mul_(1.0)  # forward / backward
            evs[2].record()
            side.wait_event(evs[2])
            with torch.cuda.stream(side):
                dist.reduce_scatter_tensor(buf, buf)
                buf.mul_(1.0)  # sumsq
            torch.cuda.current_stream().wait_stream(side)
        elif case.startswith("side_"):
            # every collective blocking on the optimizer side stream, compute between them
            half = buf.numel() // 2
            evs[0].record()
            side.wait_event(evs[0])
            with torch.cuda.stream(side):
                if case in ("side_zero1", "side_rs_mul_ag", "side_rs_ag", "side_rs_ar_ag_sync"):
                    dist.reduce_scatter_tensor(buf, buf)
                elif case == "side_two_buckets":
                    dist.reduce_scatter_tensor(buf[:half], buf[:half])
                if case in ("side_zero1", "side_rs_mul_ag", "side_ar_mul_ag"):
                    buf.mul_(1.0)
                if case in ("side_zero1", "side_ar_mul_ag", "side_rs_ar_ag_sync"):
                    dist.all_reduce(tot1)
                if case in ("side_zero1", "side_rs_mul_ag", "side_ar_mul_ag"):
                    buf.mul_(1.0)
            if case == "side_two_buckets":
                buf[half:].mul_(1.0)  # compute stream: the next bucket's gradient
                evs[1].record()
                side.wait_event(evs[1])
                with torch.cuda.stream(side):
                    dist.reduce_scatter_tensor(buf[half:], buf[half:])
                    dist.all_reduce(tot1)
                    buf[:half].mul_(1.0)
                    dist.all_gather_into_tensor(buf[:half], buf[:half])
                    evs[2].record()
                    buf[half:].mul_(1.0)
                    dist.all_gather_into_tensor(buf[half:], buf[half:])
                    evs[3].record()
                torch.cuda.current_stream().wait_event(evs[2])
                torch.cuda.current_stream().wait_event(evs[3])
            else:
                with torch.cuda.stream(side):
                    dist.all_gather_into_tensor(buf, buf)
                    evs[3].record()
                torch.cuda.current_stream().wait_event(evs[3])
            torch.cuda.current_stream().wait_stream(side)
        elif case.startswith("comm_stream"):
            # the round-6 GradReducer / FlatAdamW structure: blocking collectives on a comm stream,
            # ordered by events against the compute (capture) stream and the optimizer side stream
            anc = case.endswith("_anchor")  # a one-element kernel before each collective: the
            # issuing stream's capture dependencies become ONE node
            evs[0].record()
            comm.wait_event(evs[0])
            with torch.cuda.stream(comm):
                if anc:
                    anchor.zero_()
                dist.reduce_scatter_tensor(buf, buf)
                evs[1].record()
            side.wait_event(evs[1])
            with torch.cuda.stream(side):
                if not case.startswith("comm_stream_rs_ag"):
                    torch.sum(buf[:8], dim=0, keepdim=True, out=tot1)
                    if anc:
                        anchor.zero_()
                    dist.all_reduce(tot1)
                buf.mul_(1.0)
                evs[2].record()
            if case != "comm_stream_rs_ar":
                comm.wait_event(evs[2])
                with torch.cuda.stream(comm):
                    if anc:
                        anchor.zero_()
                    dist.all_gather_into_tensor(buf, buf)
                    evs[3].record()
                torch.cuda.current_stream().wait_event(evs[3])
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.current_stream().wait_stream(comm)
        elif case == "rs_then_ag_side":
            w = dist.reduce_scatter_tensor(buf, buf, async_op=True)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                w.wait()
                g = dist.all_gather_into_tensor(buf, buf, async_op=True)
            g.wait()
            torch.cuda.current_stream().wait_stream(side)
        elif case == "two_async_side":
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                a1 = dist.all_reduce(buf[:1], async_op=True)
                a2 = dist.all_gather_into_tensor(buf, buf, async_op=True)
                a1.wait()
            a2.wait()
            torch.cuda.current_stream().wait_stream(side)
        elif case == "ar_clone_side":
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                tot = buf[:1].clone()
                dist.all_reduce(tot)
            torch.cuda.current_stream().wait_stream(side)
        elif case == "zero1_no_clone":
            w = dist.reduce_scatter_tensor(buf, buf, async_op=True)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                w.wait()
                dist.all_reduce(other[:1])
                buf.mul_(1.0)
                g = dist.all_gather_into_tensor(buf, buf, async_op=True)
            g.wait()
            torch.cuda.current_stream().wait_stream(side)
        elif case in ("zero1_gate_wait_on_side", "zero1_async_norm"):
            w = dist.reduce_scatter_tensor(buf, buf, async_op=True)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                w.wait()
                tot = buf[:1].clone()
                if case == "zero1_async_norm":
                    dist.all_reduce(tot, async_op=True).wait()
                else:
                    dist.all_reduce(tot)
                buf.mul_(1.0)
                g = dist.all_gather_into_tensor(buf, buf, async_op=True)
                if case == "zero1_gate_wait_on_side":
                    g.wait()
            if case == "zero1_async_norm":
                g.wait()
            torch.cuda.current_stream().wait_stream(side)
        else:
            raise SystemExit(f"unknown case {case}")
        buf.add_(1.0)

    body()  # eager warm-up (communicator, streams)
    torch.cuda.synchronize()
    before = float(buf[5].item())
    g = torch.cuda.CUDAGraph()
    print(f"[{case}] capturing", flush=True)
    with torch.cuda.graph(g):
        body()
    print(f"[{case}] captured; replaying", flush=True)
    KEEP.clear()
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    after = float(buf[5].item())
    print(f"[{case}] OK before={before} after={after} (+2 expected)", flush=True)
    del g
    dist.destroy_process_group()
    del cur, other


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="")
    ap.add_argument("--only", default="", help="comma-separated cases (default: all)")
    ap.add_argument("--env", action="append", default=[], help="K=V set in every child")
    a = ap.parse_args()
    if a.case:
        child(a.case)
        return 0
    worst = 0
    for c in (a.only.split(",") if a.only else CASES):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), RANK="0", WORLD_SIZE="1",
                   LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
        env.update(kv.split("=", 1) for kv in a.env)
        r = subprocess.run([sys.executable, "-X", "faulthandler", __file__, "--case", c], env=env,
                           capture_output=True, text=True, timeout=120)
        tail = "\n".join((r.stdout + r.stderr).strip().splitlines()[-25:])
        print(f"=== {c} {' '.join(a.env)}: rc {r.returncode}\n{tail}\n", flush=True)
        if r.returncode != 0:
            worst = 1
    return worst


if __name__ == "__main__":
    sys.exit(main())
