"""Fault-tolerant training loop (the reference's ``train.py``, MI355X-first).

Observable behaviour follows reference ``train.py:12-134`` — same flags, same
log lines, same checkpoint file and keys, same exit policy
(``ft.exit_handler``), exit code 0 on every path — with the reference's
hazards fixed:

* signals are flags polled at step boundaries (``ft.signals``), agreed across
  data-parallel ranks with a 4-byte MAX vote, then raised as
  :class:`SignalInterrupt` into the reference's single ``except`` → handler;
  a step is therefore never torn, and ``training_step`` in a checkpoint is
  always the index of the next batch to run (§A.3);
* the injected fault (``--raise-error --error-step N``) fires at the start of
  step N, before any of its work, so "Checkpoint saved at step N" and the
  resumed run replays batch N exactly once;
* gradient clipping really clips (§A.1), resume loads strictly (§A.2), the
  run is seeded (§A.4), the data position is restored in O(1) (§A.7) and the
  model is initialised on the device (§A.8);
* checkpoints are written by the asynchronous engine (``ckpt.engine``) —
  periodic saves (``--save-every``) overlap training; exit saves block until
  the file is durable.

Compute runs through the flat-buffer model (``models.llama``) with the gfx950
HIP kernels, bucketed RCCL all-reduce overlapped with backward
(``parallel.ddp``) and the fused clip+AdamW kernels (``optim.adamw``).
"""
from __future__ import annotations

import json
import os
import sys
import time
from typing import Any, Dict, Optional

import torch

from .ckpt.engine import CheckpointEngine
from .ckpt.format import checkpoint_file, load_checkpoint
from .ckpt.state import build_checkpoint, capture_rng, restore_model, restore_rng, shard_regions
from .data.loader import IterableSource, MapSource, SyntheticSource, TrainLoader
from .data.synthetic import SyntheticTokens
from .ft.exit_handler import classify_exception, handle_exit
from .ft.signals import SignalInterrupt, SignalMonitor
from .models.llama import build_model, flops_per_token, model_args_for
from .optim.adamw import FlatAdamW
from .parallel import dist as fdist
from .parallel.ddp import GradReducer
from .utils.config import PRECISION_STR_TO_DTYPE, get_args, jobid
from .utils.logging import init_logger, logger
from .utils.lr import build_lr_scheduler

SYNTHETIC_VOCAB = 131072  # the reference's Mistral-Nemo tokenizer size


class InjectedFault(Exception):
    """``--raise-error`` fault (reference train.py:112-113; same message and args)."""

    def __init__(self):
        super().__init__("Simulated exception to test signal handler", -1)


class _LossLog:
    """Deferred step logging without host stalls.

    At a log step the loss is copied D2H into pinned memory and a timing event is
    recorded on the compute stream; the line is printed at a later step boundary
    once the event has completed. Step time is the GPU time between consecutive
    log events (the host runs ahead of the GPU, so host timestamps would measure
    enqueue time, not step time).
    """

    def __init__(self, device: torch.device, tokens_per_step: int, world: int, flops_per_token: float):
        self.cuda = device.type == "cuda"
        self.pending = []  # (step, host loss, event, extra)
        self.tokens = tokens_per_step
        self.world = world
        self.fpt = flops_per_token
        self.last = None  # (step, event or host time)

    def mark(self):
        """Timing origin (call once the first step is enqueued)."""
        self.last = None

    def push(self, step: int, loss: torch.Tensor, extra: Dict[str, Any], norm=None):
        """``norm``: optional (device tensor, event) of the step's gradient norm (logged as grad_norm)."""
        vals = [loss.detach().float().reshape(1)]
        if norm is not None:
            if self.cuda and norm[1] is not None:
                torch.cuda.current_stream().wait_event(norm[1])  # the norm is finished on the optimizer stream
            vals.append(norm[0].detach().float().reshape(1))
        if self.cuda:
            h = torch.empty(len(vals), dtype=torch.float32, pin_memory=True)
            h.copy_(torch.cat(vals), non_blocking=True)
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self.pending.append((step, h, ev, extra))
        else:
            self.pending.append((step, torch.cat(vals), time.perf_counter(), extra))

    def flush(self, force: bool = False):
        keep = []
        for step, h, ev, extra in self.pending:
            if self.cuda and not force and not ev.query():
                keep.append((step, h, ev, extra))
                continue
            if self.cuda:
                ev.synchronize()
            hv = h.tolist()
            msg = f"Training step: {step} | Loss: {hv[0]:.2f}"
            if len(hv) > 1:
                extra = dict(extra)
                extra["grad_norm"] = f"{hv[1]:.3f}"
            if self.last is not None:
                ls, lev = self.last
                dt = (lev.elapsed_time(ev) / 1e3) if self.cuda else (ev - lev)
                dt /= max(1, step - ls)
                tok_s = self.tokens / dt
                extra = dict(extra)
                extra["step_ms"] = f"{dt * 1e3:.1f}"
                extra["tok/s"] = f"{tok_s:.0f}"
                if self.cuda:
                    extra["MFU"] = f"{tok_s / self.world * self.fpt / 2.5e15:.3f}"
            self.last = (step, ev)
            if extra:
                msg += " | " + " | ".join(f"{k}: {v}" for k, v in extra.items())
            logger.info(msg)
        self.pending = keep


def _build_source(args, info, tokenizer_vocab_holder: Dict[str, Any]):
    B, S = args.batch_size, args.sequence_length
    if args.synthetic_data:
        vocab = args.vocab_size or SYNTHETIC_VOCAB
        tokenizer_vocab_holder["vocab"] = vocab
        ds = SyntheticTokens(vocab, S, seed=args.seed, rank=info.rank, world_size=info.world_size, pin=False)
        return SyntheticSource(ds, B)
    from .data.parquet import CollatorForCLM, IterableParquetDataset, ParquetDataset
    from .data.tokenizer import load_tokenizer, pad_token_id

    tok = load_tokenizer(args.tokenizer_name_or_path)
    tokenizer_vocab_holder["vocab"] = args.vocab_size or int(tok.vocab_size)
    if args.iterable_dataset:
        bos = getattr(tok, "bos_token_id", None)
        ds = IterableParquetDataset(args.dataset, tok, S, bos_token_id=1 if bos is None else int(bos),
                                    rank=info.rank, world_size=info.world_size)
        return IterableSource(ds, B)
    ds = ParquetDataset(args.dataset, tok, S, B * args.training_steps * info.world_size)
    return MapSource(ds, CollatorForCLM(S, pad_token_id(tok)), B, info.rank, info.world_size)


def train(args) -> int:
    t_setup = time.perf_counter()
    info = fdist.init_distributed(args.device)
    init_logger(info.rank)
    logger.info(f"Experiment args: {args}")
    # Install the flag handlers before any slow setup: a signal that arrives while
    # the checkpoint or the model is loading is acted on at the first step
    # boundary instead of killing the job (the reference registers after setup,
    # train.py:89-90).
    monitor = SignalMonitor().install()
    device = info.device
    model_dtype = PRECISION_STR_TO_DTYPE[args.model_dtype]
    if device.type == "cuda" and model_dtype != torch.bfloat16:
        raise ValueError("the gfx950 kernels are bf16; use --model-dtype bf16 on the GPU (any dtype on --device cpu)")
    torch.manual_seed(args.seed)
    from .ops.attention import set_deterministic

    set_deterministic(args.flash_bwd == "deterministic")
    job_id = jobid()

    checkpoint = None
    if args.checkpoint_id:
        logger.info(f"Loading checkpoint from {args.checkpoint_path}")
        checkpoint = load_checkpoint(checkpoint_file(args.checkpoint_path, args.checkpoint_id))

    logger.info("Setting up DataLoaders...")
    holder: Dict[str, Any] = {}
    source = _build_source(args, info, holder)
    loader_state = None
    if checkpoint is not None:
        dl = checkpoint.get("data_loader")
        if isinstance(dl, list):
            if len(dl) == info.world_size:
                loader_state = dl[info.rank]
            elif source.kind == "iterable":
                raise ValueError(f"checkpoint has data-loader states for {len(dl)} ranks, this run has "
                                 f"{info.world_size}; the packing dataset cannot be re-sharded")
            else:
                logger.warning(f"checkpoint was written by {len(dl)} ranks, resuming on {info.world_size}: "
                               "data order restarts from the global step index")
        elif isinstance(dl, dict):
            loader_state = dl
    start_step = int(checkpoint["training_step"]) if checkpoint is not None else 0
    if loader_state is not None and int(loader_state.get("next_step", start_step)) != start_step:
        raise ValueError("data-loader state does not match training_step in the checkpoint")
    loader = TrainLoader(source, start_step=start_step, state=loader_state, prefetch=args.prefetch)

    logger.info("Setting up Model...")
    margs = model_args_for(args.model, vocab_size=holder["vocab"], seq_len=args.sequence_length)
    model = build_model(margs, device, model_dtype, seed=args.seed)
    if args.activation_checkpointing:
        model.set_activation_checkpointing(args.activation_checkpointing)
        logger.info(f"Activation checkpointing: recomputing {model.recompute_layers} of {model.n_layers} blocks")
    if checkpoint is not None:
        restore_model(model, checkpoint["model"])
        logger.info("Model loaded from checkpoint")
    if args.compile:
        logger.info("`--compile`: not using torch.compile — the step already runs fused gfx950 kernels "
                    "(flag accepted for CLI compatibility)")
    model.train()

    state_dtype = PRECISION_STR_TO_DTYPE[args.optimizer_state_dtype] if args.optimizer_state_dtype else None
    reducer = GradReducer(model.flat, model.sinks_in_backward_order(), bucket_mb=args.dp_bucket_mb,
                          mode=args.dp_mode or None)
    optimizer = FlatAdamW(model.parameters(), model.flat, lr=args.learning_rate, state_dtype=state_dtype,
                          max_grad_norm=args.grad_max_norm, fused=args.fused_optimizer, reducer=reducer)
    model.gate = optimizer.gate
    if checkpoint is not None:
        optimizer.load_state_dict(checkpoint["optimizer"])
        logger.info("Optimizer loaded from checkpoint")
    lr_scheduler = build_lr_scheduler(optimizer, args.lr_warmup_steps)
    if checkpoint is not None:
        lr_scheduler.load_state_dict(checkpoint["lr_scheduler"])
        # LambdaLR's constructor already stepped the groups back to lambda(0); the
        # reference keeps that LR for the first resumed step. Re-apply the saved one.
        for g, lr in zip(optimizer.param_groups, lr_scheduler.get_last_lr()):
            g["lr"] = lr
        logger.info("LR Scheduler loaded from checkpoint")
        restore_rng(checkpoint.get("rng"), device)
    if checkpoint is not None:
        training_step = int(checkpoint["training_step"])
        logger.info(f"Resuming training from training_step {training_step}")
    else:
        training_step = 0
        logger.info("Starting training!")
    del checkpoint
    from .ckpt.restore import release as _release_restore_ring

    _release_restore_ring()

    if info.distributed:
        if training_step == 0:
            reducer.broadcast_params()
        # every rank must agree on where it resumes
        steps = fdist.ctrl_all_gather_object(training_step)
        if len(set(steps)) != 1:
            raise RuntimeError(f"ranks disagree on training_step: {steps}")
        logger.info(f"Data parallel over {info.world_size} ranks: {reducer.summary()}")

    ckpt_path = checkpoint_file(args.checkpoint_path, job_id)
    ckpt = {"engine": None}
    # FT_SHARDED_CKPT=1 forces the multi-writer protocol on a 1-rank process group (test hook)
    sharded = info.world_size > 1 or (info.ckpt_group is not None and os.environ.get("FT_SHARDED_CKPT") == "1")

    def ckpt_engine():
        if ckpt["engine"] is None:
            if sharded:
                # every rank writes its own pieces of the one file (ZeRO-1: its AdamW shards)
                regions = shard_regions(model, optimizer, info.rank, info.world_size)
                ckpt["engine"] = CheckpointEngine(regions, mode=args.checkpoint_mode,
                                                  writer_threads=args.checkpoint_writer_threads,
                                                  group=info.ckpt_group, rank=info.rank, world=info.world_size,
                                                  sharded=True)
            else:
                ckpt["engine"] = CheckpointEngine(
                    {"params": model.flat.params, "exp_avg": optimizer.exp_avg, "exp_avg_sq": optimizer.exp_avg_sq},
                    mode=args.checkpoint_mode, writer_threads=args.checkpoint_writer_threads)
        return ckpt["engine"]

    if not args.no_checkpoint_prealloc:
        # pin the snapshot's host buffers while training starts: the first save (often the
        # SIGUSR1 one, racing the Slurm deadline) then only copies and writes
        ckpt_engine().preallocate_async()

    def save_checkpoint(blocking: bool, collective: bool = True):
        optimizer.gate.wait_all()  # the snapshot must follow this step's parameter updates
        if collective:
            states = fdist.ctrl_all_gather_object(loader.state_dict())
        else:  # rank-local save (error on this rank only): other ranks' positions unknown
            states = [None] * info.world_size
            states[info.rank] = loader.state_dict()
        step_now = training_step
        rng = capture_rng(device)

        def build(host):
            return build_checkpoint(model, optimizer, lr_scheduler, step_now, host,
                                    data_loader=states if info.distributed else states[0], rng=rng,
                                    extra_meta={"world_size": info.world_size, "job_id": str(job_id)})

        if sharded and not collective:
            if optimizer.zero1:
                logger.error("ZeRO-1 optimizer state is sharded over the ranks; a rank-local error cannot "
                             "write a complete checkpoint")
                return False
            # replicated state: this rank writes the whole file alone
            solo = CheckpointEngine({"params": model.flat.params, "exp_avg": optimizer.exp_avg,
                                     "exp_avg_sq": optimizer.exp_avg_sq}, mode="host",
                                    writer_threads=args.checkpoint_writer_threads)
            return solo.save(ckpt_path, build, step=step_now, blocking=True)
        engine = ckpt_engine()
        writes = sharded or info.is_main
        st = engine.save(ckpt_path, build, step=step_now, blocking=blocking) if writes else None
        if collective and blocking:
            fdist.barrier()
        return st

    metrics_f = open(args.metrics_file, "a") if (args.metrics_file and info.is_main) else None
    B, S, W = args.batch_size, args.sequence_length, info.world_size
    fpt = flops_per_token(margs, S)
    losslog = _LossLog(device, B * S * W, W, fpt)
    synthetic_counts = args.synthetic_data  # no ignore_index labels: the global count is static
    inv_static = None
    if synthetic_counts:
        inv_static = torch.full((1,), 1.0 / (B * S * W), dtype=torch.float32, device=device)
    t_window, steps_window = time.perf_counter(), 0
    logger.info(f"Setup took {time.perf_counter() - t_setup:.2f}s")
    prof, prof_range = None, None
    if args.profile_steps:
        a0, a1 = (int(v) for v in args.profile_steps.split(":"))
        prof_range = (a0, a1)

    try:
        while training_step < args.training_steps:
            if args.raise_error and training_step == args.error_step:
                raise InjectedFault()
            if prof_range is not None and training_step == prof_range[0] and prof is None:
                acts = [torch.profiler.ProfilerActivity.CPU]
                if device.type == "cuda":
                    acts.append(torch.profiler.ProfilerActivity.CUDA)
                prof = torch.profiler.profile(activities=acts, record_shapes=True)
                prof.__enter__()
            batch = next(loader)
            tok = batch.inputs.to(device, non_blocking=True)
            lab = batch.labels.to(device, non_blocking=True)
            if inv_static is not None:
                inv = inv_static
            else:
                cnt = torch.tensor([float(batch.num_items)], dtype=torch.float32)
                cnt = cnt.to(device, non_blocking=True)
                if info.distributed:
                    torch.distributed.all_reduce(cnt)
                inv = cnt.clamp_min(1.0).reciprocal()
            loss = model(tok, lab, inv)
            loss.backward()
            reducer.finish()
            optimizer.clip_grad_norm_(args.grad_max_norm)
            if ckpt["engine"] is not None:
                ckpt["engine"].fence()
            lr_now = optimizer.param_groups[0]["lr"]
            optimizer.step()
            lr_scheduler.step()
            steps_window += 1

            if training_step == 1 or training_step % args.logging_frequency == 0:
                extra = {"lr": f"{lr_now:.3e}"}
                if device.type == "cuda":
                    extra["peak_HBM_GB"] = f"{torch.cuda.max_memory_allocated(device) / 2**30:.1f}"
                if info.distributed:
                    # each rank's loss is its token sum over the GLOBAL token count: the
                    # logged global-batch mean is their sum (every rank logs at the same steps)
                    loss = loss.detach().clone()
                    torch.distributed.all_reduce(loss)
                losslog.push(training_step, loss, extra, norm=optimizer.norm_for_logging())
                if metrics_f is not None:
                    now = time.perf_counter()
                    dt = (now - t_window) / max(1, steps_window)
                    metrics_f.write(json.dumps({"step": training_step, "host_step_ms": dt * 1e3}) + "\n")
                    metrics_f.flush()
                    t_window, steps_window = now, 0
            training_step += 1
            if prof is not None and training_step >= prof_range[1]:
                if device.type == "cuda":
                    torch.cuda.synchronize()
                prof.__exit__(None, None, None)
                os.makedirs(args.profile_dir, exist_ok=True)
                out = os.path.join(args.profile_dir, f"trace_rank{info.rank}_steps{prof_range[0]}-{prof_range[1]}.json")
                prof.export_chrome_trace(out)
                logger.info(f"torch.profiler trace written to {out}")
                prof, prof_range = None, None
            losslog.flush()
            optimizer.check_finite(block=False)  # deferred non-finite check → error path
            done = ckpt["engine"].poll() if ckpt["engine"] is not None else None
            if done is not None:
                logger.info(f"Checkpoint written: {done.path} ({done.bytes / 1e9:.2f} GB, "
                            f"stall {done.stall_s:.3f}s, durable after {done.total_s:.2f}s)")
            if args.save_every and training_step % args.save_every == 0 and training_step < args.training_steps:
                save_checkpoint(blocking=args.no_async_checkpoint)
            if args.consensus_every <= 1 or training_step % args.consensus_every == 0:
                sig = monitor.pending()
                if info.distributed:
                    sig = fdist.ctrl_allreduce_max(sig)
                if sig:
                    raise SignalInterrupt(sig)
        losslog.flush(force=True)
        if device.type == "cuda":
            torch.cuda.synchronize()
        optimizer.check_finite(block=True)
        if ckpt["engine"] is not None:
            ckpt["engine"].wait()
        logger.info("Training completed")
    except Exception as e:  # noqa: BLE001 - the reference catches everything here (train.py:121)
        losslog.flush(force=True)
        exit_type = classify_exception(e)
        if exit_type == -1 and not isinstance(e, InjectedFault):
            logger.error(f"Training error: {e!r}")
        # signals are agreed across ranks; the injected fault fires on every rank at
        # the same step; any other error may be local to this rank
        collective = info.distributed and isinstance(e, (SignalInterrupt, InjectedFault))
        try:
            if ckpt["engine"] is not None:
                ckpt["engine"].wait()
        except Exception as we:  # noqa: BLE001
            logger.error(f"previous checkpoint write failed: {we!r}")

        def _save():
            with monitor.blocked():
                st = save_checkpoint(blocking=True, collective=collective or not info.distributed)
            if st is False:
                return False
            if st is not None:
                logger.info(f"Checkpoint {st.path}: {st.bytes / 1e9:.2f} GB in {st.total_s:.2f}s "
                            f"(mode {st.mode})")

        handle_exit(_save, training_step, exit_type, logger, job_id=job_id,
                    sbatch_script=args.sbatch_script, is_main=info.is_main)
    finally:
        loader.close()
        if metrics_f is not None:
            metrics_f.close()
        monitor.uninstall()
    sys.stdout.flush()
    sys.stderr.flush()
    return 0


def main(argv=None) -> None:
    args = get_args(argv)
    rc = train(args)
    fdist.destroy()
    sys.exit(rc)


if __name__ == "__main__":
    main()
