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

import collections
import json
import os
import signal
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
from .optim.adamw import FlatAdamW, NonFiniteGradError, nonfinite_message
from .parallel import dist as fdist
from .parallel.ddp import GradReducer
from .utils.config import PRECISION_STR_TO_DTYPE, get_args, jobid
from .utils.logging import init_logger, logger
from .utils.lr import build_lr_scheduler, rollback_lr_scheduler

SIGTERM_NUM = int(signal.SIGTERM)
SYNTHETIC_VOCAB = 131072  # the reference's Mistral-Nemo tokenizer size
DP_DEFAULT_SAVE_EVERY = 200  # --save-every when unset and world > 1 (BASELINE config 3)


class InjectedFault(Exception):
    """``--raise-error`` fault (reference train.py:112-113; same message and args)."""

    def __init__(self):
        super().__init__("Simulated exception to test signal handler", -1)


class _LossLog:
    """Step logging without host stalls, summed over data-parallel ranks.

    At a log step the loss (and grad norm) is copied D2H into pinned memory behind
    an event on the compute stream. Two step boundaries later — when that copy has
    long landed — :meth:`take` hands the entry to the trainer, which adds the local
    value to the per-step vote; the vote returns the ranks' sum (each rank's loss
    is its token sum over the GLOBAL token count, so the sum is the global-batch
    mean) and :meth:`emit` prints the reference's line. No data-plane collective and
    no device sync is needed for logging. Step time is the GPU time between
    consecutive log events (the host runs ahead of the GPU).
    """

    def __init__(self, device: torch.device, tokens_per_step: int, world: int, flops_per_token: float,
                 peak_flops: float = 2.5e15):
        self.cuda = device.type == "cuda"
        self.pending = []  # [step, host values, event or host time, extra]
        self.tokens = tokens_per_step
        self.world = world
        self.fpt = flops_per_token
        self.peak = peak_flops  # the model dtype's dense matrix-core peak (models.llama.PEAK_FLOPS)
        self.last = None  # (step, event or host time)

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
            self.pending.append([step, h, ev, extra])
        else:
            self.pending.append([step, torch.cat(vals), time.perf_counter(), extra])

    def take(self, upto: int):
        """Entries of steps <= ``upto`` (host values ready; blocks on their copies)."""
        out = [e for e in self.pending if e[0] <= upto]
        self.pending = [e for e in self.pending if e[0] > upto]
        for e in out:
            if self.cuda:
                e[2].synchronize()
            e[1] = e[1].tolist()
        return out

    def emit(self, e, loss: float) -> None:
        step, hv, ev, extra = e
        msg = f"Training step: {step} | Loss: {loss:.2f}"
        extra = dict(extra)
        if len(hv) > 1:
            extra["grad_norm"] = f"{hv[1]:.3f}"
        if self.last is not None and step > self.last[0]:
            ls, lev = self.last
            dt = (lev.elapsed_time(ev) / 1e3) if self.cuda else (ev - lev)
            dt /= max(1, step - ls)
            tok_s = self.tokens / dt
            extra["step_ms"] = f"{dt * 1e3:.1f}"
            extra["tok/s"] = f"{tok_s:.0f}"
            if self.cuda:
                extra["MFU"] = f"{tok_s / self.world * self.fpt / self.peak:.3f}"
        self.last = (step, ev)
        if extra:
            msg += " | " + " | ".join(f"{k}: {v}" for k, v in extra.items())
        logger.info(msg)

    def drop_after(self, step: int) -> None:
        """Forget entries of rolled-back steps."""
        self.pending = [e for e in self.pending if e[0] < step]


class _StopTraining(Exception):
    """Raised at a step boundary once every rank has agreed to stop (carries the exit cause)."""

    def __init__(self, cause: BaseException):
        super().__init__(repr(cause))
        self.cause = cause


class _GraphDone(Exception):
    """Internal: the step ran as a graph replay (skips the eager compute block)."""


class _FatalStepError(Exception):
    """A failure left this rank unable to finish its share of the step's collectives."""


class _RankFault:
    """Rank-local fault injection for the DP tests: ``FT_INJECT_FAULT=rank:step:phase``.

    Phases: ``data`` (OSError while fetching the batch), ``forward``, ``backward`` (OSError
    raised inside backward after the first gradient bucket was launched), ``optimizer``
    (before ``optimizer.step()``), ``post`` (after the step), ``kill`` (SIGKILL itself),
    ``hang`` (sleep forever) at the start of the step, and ``peerloss`` (the step's boundary vote
    raises :class:`PeerFailure`, as when a peer died). Under the whole-step HIP graph the
    forward / backward / optimizer faults fire before the replay, which then runs poisoned."""

    def __init__(self, spec: str, rank: int):
        self.step = self.phase = None
        if spec:
            r, st, ph = spec.split(":")
            if int(r) == rank:
                self.step, self.phase = int(st), ph

    def at(self, step: int, phase: str) -> bool:
        return self.step == step and self.phase == phase

    def fire(self, step: int, phase: str) -> None:
        if not self.at(step, phase):
            return
        if phase == "kill":
            os.kill(os.getpid(), signal.SIGKILL)
        if phase == "hang":
            while True:
                time.sleep(1)
        raise OSError(5, f"injected I/O error on this rank at step {step} ({phase})")


def _build_source(args, info, tokenizer_vocab_holder: Dict[str, Any]):
    # one loader batch = the K micro-batches of one optimizer step (gradient accumulation)
    B, S = args.batch_size * max(1, int(args.grad_accum)), args.sequence_length
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
    if args.compile or args.hip_graph:
        fdist.graph_capture_env()
    info = fdist.init_distributed(args.device, peer_timeout_s=args.peer_timeout)
    init_logger(info.rank)
    logger.info(f"Experiment args: {args}")
    # Install the flag handlers before any slow setup: a signal that arrives while
    # the checkpoint or the model is loading is acted on at the first step
    # boundary instead of killing the job (the reference registers after setup,
    # train.py:89-90).
    monitor = SignalMonitor().install()
    device = info.device
    model_dtype = PRECISION_STR_TO_DTYPE[args.model_dtype]
    if device.type == "cuda" and model_dtype == torch.float64:
        # the reference builds the model in fp64 on the GPU too (utils.py:14-19, train.py:54-59); the
        # gfx950 kernels cover bf16 / fp16 / fp32, so fp64 tensors take the composed-PyTorch path
        # (rocBLAS dgemm, reference attention): correct, not fast
        logger.info("--model-dtype fp64 on the GPU: composed PyTorch ops (the HIP kernels cover bf16/fp16/fp32)")
    if model_dtype == torch.float32:
        # the reference accepts fp32 (utils.py:14-19); the w4 GEMM is 16-bit, so an fp32 model's GEMMs
        # take the fp32 MFMA kernel (ops/functional.py f32_route; tests/test_routing_cpu.py)
        logger.info("--model-dtype fp32: GEMMs on the fp32 MFMA kernel (gemm_f32, v_mfma_f32_16x16x4_f32; "
                    "hipBLASLt where K % 32 != 0) -- the w4 GEMM is bf16/fp16; norms, RoPE, SwiGLU, attention, "
                    "cross-entropy and AdamW run their fp32 HIP kernels")
    torch.manual_seed(args.seed)
    from .ops.attention import set_deterministic

    set_deterministic(args.flash_bwd == "deterministic")
    job_id = jobid()

    checkpoint = None
    resume_file = None  # the file this job resumed from (--prune-consumed deletes it later)
    if args.checkpoint_id:
        dirs = [args.checkpoint_path] + ([args.checkpoint_alt_path] if args.checkpoint_alt_path else [])
        cands = [checkpoint_file(d_, args.checkpoint_id) for d_ in dirs]
        resume_file = next((c for c in cands if os.path.exists(c)), cands[0])
        logger.info(f"Loading checkpoint from {os.path.dirname(resume_file) or args.checkpoint_path}")
        checkpoint = load_checkpoint(resume_file)

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
    if loader_state is not None:
        logger.info(f"Data loader position restored: {loader_state}")

    logger.info("Setting up Model...")
    margs = model_args_for(args.model, vocab_size=holder["vocab"], seq_len=args.sequence_length)
    model = build_model(margs, device, model_dtype, seed=args.seed)
    if args.activation_checkpointing:
        model.set_activation_checkpointing(args.activation_checkpointing,
                                           recompute_attention=getattr(args, "recompute_attention", False))
        logger.info(f"Activation checkpointing: recomputing {model.recompute_layers} of {model.n_layers} blocks")
    if checkpoint is not None:
        restore_model(model, checkpoint["model"])
        logger.info("Model loaded from checkpoint")
    if args.compile:
        # The reference compiles the model (train.py:61-63) to cut launch overhead and fuse ops.
        # Here the ops are already fused gfx950 kernels; what is left to "compile" is the launch
        # sequence, and the MI355X-native form of that is the whole-step HIP graph (--hip-graph):
        # on GPU ranks without gradient accumulation --compile turns it on (under DP -- ZeRO-1 or
        # all-reduce -- the bucket collectives and ZeRO-1's parameter all-gathers are captured into
        # the graph; the per-step vote stays on the host, between replays). Host-side accumulation
        # or the fp64 path cannot be captured: there the flag is accepted and logged as not applied.
        from .graphs import hw_queue_problem

        graphable = model_dtype in (torch.bfloat16, torch.float16, torch.float32) and not hw_queue_problem()
        if device.type == "cuda" and max(1, int(args.grad_accum)) == 1 and graphable:
            logger.info("Using `torch.compile`")
            logger.info("`torch.compile` -> whole-step HIP graph capture (--hip-graph): the step's "
                        "kernel launches are recorded once and replayed")
            args.hip_graph = True
        else:
            logger.info("Using `torch.compile` — accepted for CLI compatibility, not applied: the step "
                        "already runs fused gfx950 kernels and the whole-step HIP graph needs GPU ranks "
                        "without gradient accumulation, in a dtype the HIP kernels run (bf16/fp16/fp32: "
                        "the fp64 composed path synchronises with the host inside the step)"
                        + ("; " + hw_queue_problem() if hw_queue_problem() else ""))
    model.train()

    # AdamW moments default to the model dtype like the reference, except under fp16: the second
    # moment g^2 of typical gradients (1e-4 .. 1e-3) is below fp16's normal range, flushes to 0 and
    # the update m / (sqrt(v) + eps) explodes within a few steps (the tiny preset diverges at step 5
    # with fp16 moments, on the CPU path too); fp32 moments keep fp16 training stable.
    if args.optimizer_state_dtype:
        state_dtype = PRECISION_STR_TO_DTYPE[args.optimizer_state_dtype]
    else:
        state_dtype = torch.float32 if model_dtype == torch.float16 else None
    reducer = GradReducer(model.flat, model.sinks_in_backward_order(), bucket_mb=args.dp_bucket_mb,
                          mode=args.dp_mode or None, reduce_dtype=args.dp_reduce_dtype)
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
    # loader position before each step (what a checkpoint taken at that step boundary records)
    loader_at: Dict[int, Any] = {}

    def log_digest(step: int, when: str = "") -> None:
        """--state-digest: an order-independent digest of params / moments + the loader position,
        comparable across a save (exit handler) and the resume from it, or across two runs."""
        if not getattr(args, "state_digest", False):
            return
        from .utils.digest import state_digest

        dg = state_digest(model.flat.params, optimizer.exp_avg, optimizer.exp_avg_sq)
        # the loader position a checkpoint at this step boundary records (the live loader may
        # already have fetched the next batch when a signal stops the run)
        pos = loader_at.get(step, loader.state_dict())
        logger.info(f"[rank {info.rank}] State digest at step {step}{when}: params={dg['params']} "
                    f"exp_avg={dg['exp_avg']} exp_avg_sq={dg['exp_avg_sq']} "
                    f"optimizer_step={optimizer.step_count} data_loader={json.dumps(pos, sort_keys=True)}")

    if checkpoint is not None:
        training_step = int(checkpoint["training_step"])
        logger.info(f"Resuming training from training_step {training_step}")
        log_digest(training_step, " (resumed)")
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

    save_dir = args.checkpoint_path
    if args.checkpoint_alt_path and resume_file is not None and \
            os.path.realpath(os.path.dirname(resume_file)) == os.path.realpath(args.checkpoint_path):
        save_dir = args.checkpoint_alt_path  # rotate: never overwrite or crowd out the file resumed from
    ckpt_path = checkpoint_file(save_dir, job_id)
    if args.checkpoint_alt_path:
        logger.info(f"Checkpoints of this job go to {save_dir}")
    ckpt = {"engine": None}

    def prune_consumed() -> None:
        """--prune-consumed: this job's own checkpoint is durable; the one it resumed from goes."""
        nonlocal resume_file
        if not (args.prune_consumed and info.is_main and resume_file is not None):
            return
        if os.path.realpath(resume_file) == os.path.realpath(ckpt_path):
            return
        try:
            os.remove(resume_file)
            logger.info(f"Deleted the consumed checkpoint {resume_file} (this job's {ckpt_path} is durable)")
        except FileNotFoundError:
            pass
        resume_file = None
    # periodic saves: on by default under data parallelism (BASELINE config 3 cadence), so a
    # lost rank (OOM-kill, node failure) costs at most that many steps — ZeRO-1 survivors
    # cannot write its optimizer shards (reference train.py:121-129 saves on every path it sees)
    save_every = args.save_every if args.save_every >= 0 else (DP_DEFAULT_SAVE_EVERY if info.world_size > 1 else 0)
    if save_every and info.world_size > 1:
        logger.info(f"Periodic checkpoint every {save_every} steps")
    durable = {"step": None, "path": None}  # last checkpoint known to be on disk (this job)
    if info.is_main:
        try:  # a previous job's peer-loss lock (same job id on requeue) would block the next solo save
            os.unlink(ckpt_path + ".solo")
        except FileNotFoundError:
            pass
    sharded = info.world_size > 1

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


    def save_checkpoint(blocking: bool, step_now: int):
        """Collective save of the state at step boundary ``step_now`` (every rank calls it)."""
        optimizer.gate.wait_all()  # the snapshot must follow this step's parameter updates
        states = fdist.ctrl_all_gather_object(loader_at.get(step_now, loader.state_dict()))
        rng = capture_rng(device)

        def build(host):
            return build_checkpoint(model, optimizer, lr_scheduler, step_now, host,
                                    data_loader=states if info.distributed else states[0], rng=rng,
                                    extra_meta={"world_size": info.world_size, "job_id": str(job_id)})

        engine = ckpt_engine()
        writes = sharded or info.is_main
        st = engine.save(ckpt_path, build, step=step_now, blocking=blocking) if writes else None
        if blocking:
            fdist.barrier()
        return st

    def save_solo(step_now: int):
        """Peer lost: one surviving rank writes the whole (replicated) state alone. Returns
        False when this rank cannot (sharded optimizer state, incomplete state, another
        survivor already writing)."""
        if optimizer.zero1 or source.kind == "iterable":
            logger.error("[EXIT HANDLER] optimizer or data-loader state is sharded over the ranks; "
                         "no complete checkpoint can be written without the lost peer")
            return False
        os.makedirs(os.path.dirname(ckpt_path) or ".", exist_ok=True)
        try:  # first survivor wins; the others leave the file to it
            os.close(os.open(ckpt_path + ".solo", os.O_CREAT | os.O_EXCL | os.O_WRONLY, 0o644))
        except FileExistsError:
            logger.info("[EXIT HANDLER] another surviving rank is writing the checkpoint")
            return None
        me = loader_at.get(step_now, loader.state_dict())
        states = [dict(me) for _ in range(info.world_size)]  # stateless sources: same next_step everywhere
        rng = capture_rng(device)

        def build(host):
            return build_checkpoint(model, optimizer, lr_scheduler, step_now, host,
                                    data_loader=states if info.distributed else states[0], rng=rng,
                                    extra_meta={"world_size": info.world_size, "job_id": str(job_id)})

        solo = CheckpointEngine({"params": model.flat.params, "exp_avg": optimizer.exp_avg,
                                 "exp_avg_sq": optimizer.exp_avg_sq}, mode="host",
                                writer_threads=args.checkpoint_writer_threads)
        # (the lock file stays: a slower survivor must not write the file a second time)
        return solo.save(ckpt_path, build, step=step_now, blocking=True)

    metrics_f = open(args.metrics_file, "a") if (args.metrics_file and info.is_main) else None
    B, S, W = args.batch_size, args.sequence_length, info.world_size
    K = max(1, int(args.grad_accum))
    fpt = flops_per_token(margs, S)
    from .models.llama import PEAK_FLOPS

    losslog = _LossLog(device, B * K * S * W, W, fpt, PEAK_FLOPS.get(model_dtype, 2.5e15))
    synthetic_counts = args.synthetic_data  # no ignore_index labels: the global count is static
    inv_static = None
    if synthetic_counts:
        inv_static = torch.full((1,), 1.0 / (B * K * S * W), dtype=torch.float32, device=device)
    t_window, steps_window = time.perf_counter(), 0
    logger.info(f"Setup took {time.perf_counter() - t_setup:.2f}s")
    prof, prof_range = None, None
    if args.profile_steps:
        a0, a1 = (int(v) for v in args.profile_steps.split(":"))
        prof_range = (a0, a1)
    fault = _RankFault(os.environ.get("FT_INJECT_FAULT", ""), info.rank)
    last_save_step = training_step  # a resumed run does not re-save the state it just loaded
    # optimizer step k <-> training step k - offset (0 for fresh runs; resumed runs load both)
    offset = optimizer.step_count - training_step
    pending_err: Optional[BaseException] = None  # this rank's mid-step failure (step completed poisoned)

    def rollback_to_first_bad() -> Optional[int]:
        """Blocking check of every optimizer step so far; roll host counters back to the first
        non-finite one (its update and every later one were skipped on device)."""
        nonlocal training_step
        bad = optimizer.first_nonfinite(block=True)
        if bad is None:
            return None
        k = optimizer.step_count - bad + 1
        optimizer.rollback_steps(k)
        rollback_lr_scheduler(lr_scheduler, k)
        training_step -= k
        losslog.drop_after(training_step)
        return training_step

    def boundary(final: bool = False, save_due: bool = False) -> None:
        """Step boundary: one vote over every rank (signal, local error, lagged non-finite check,
        token count of the next batch, losses to log), then either go on or stop together.

        ``save_due``: a periodic checkpoint follows if the vote passes. Its non-finite check
        then covers every optimizer step so far (blocking), so the file never records steps
        whose updates the device guard skipped."""
        nonlocal pending_err
        if save_due:
            complete_pending()  # graph mode: the snapshot needs the last step's optimizer update
        if fault.at(training_step, "peerloss"):  # test hook: this boundary's vote fails
            raise fdist.PeerFailure(f"injected peer loss at the boundary before step {training_step}")
        sig = monitor.pending()
        err = 1.0 if pending_err is not None else 0.0
        upto = optimizer.step_count if (final or save_due) else optimizer.step_count - 1
        bad = optimizer.first_nonfinite(upto=upto, block=True)
        entries = losslog.take(training_step - (0 if final else 2))
        vec = [float(sig), err, float(bad or 0), float(boundary.count)] + [e[1][0] for e in entries]
        table = fdist.vote(vec)
        for e, lv in zip(entries, table[:, 4:].sum(0).tolist()):
            losslog.emit(e, lv)
        boundary.count_sum = float(table[:, 3].sum())
        sig_all = int(table[:, 0].max())
        err_all = bool(table[:, 1].max() > 0)
        bad_all = bool(table[:, 2].max() > 0)
        if not (sig_all or err_all or bad_all):
            return
        # stop: every rank reached the same decision from the same table
        complete_pending()  # graph mode: the last backward's optimizer step first
        rolled = rollback_to_first_bad()
        if sig_all == SIGTERM_NUM:
            raise _StopTraining(SignalInterrupt(sig_all))
        if pending_err is not None:
            raise _StopTraining(pending_err)
        if err_all:
            raise _StopTraining(RuntimeError("a peer rank failed during training (see its log); "
                                             "stopping every rank at the same step"))
        if rolled is not None:
            raise _StopTraining(NonFiniteGradError(nonfinite_message(rolled + offset + 1)))
        raise _StopTraining(SignalInterrupt(sig_all))

    boundary.count = 0
    boundary.count_sum = 0.0
    emb_dim = margs.dim
    exit_code = 0

    graphed = None
    if args.hip_graph:
        if K > 1 or device.type != "cuda" or model_dtype not in (torch.bfloat16, torch.float16, torch.float32):
            raise ValueError("--hip-graph: --grad-accum 1, --device cuda, --model-dtype bf16/fp16/fp32")
        from .graphs import GraphedStep, hw_queue_problem

        if hw_queue_problem():
            raise ValueError("--hip-graph: " + hw_queue_problem())

        inv_dev = torch.empty(1, dtype=torch.float32, device=device)  # static input of the graph

        def _fwd_bwd(tok_, lab_):
            l_ = model(tok_, lab_, inv_dev)
            l_.backward()
            reducer.finish()
            return l_

        graphed = GraphedStep(model, reducer, optimizer, lr_scheduler, _fwd_bwd)
        logger.info("HIP graph: each step replays [optimizer(k) | forward+backward(k+1)] as one graph")

    def complete_pending():
        """Graph mode: run the last backward's optimizer step (before a checkpoint / at the end)."""
        if graphed is not None and graphed.pending:
            if ckpt["engine"] is not None:
                ckpt["engine"].fence()
            graphed.finish()

    try:
        while training_step < args.training_steps:
            # ---- step boundary: fetch the batch, then agree with every rank before any compute
            loader_at[training_step] = loader.state_dict()
            loader_at.pop(training_step - 8, None)
            batch = None
            try:
                if args.raise_error and training_step == args.error_step:
                    raise InjectedFault()
                fault.fire(training_step, "kill")
                fault.fire(training_step, "hang")
                fault.fire(training_step, "data")
                batch = next(loader)
                done = ckpt["engine"].poll() if ckpt["engine"] is not None else None
                if done is not None:
                    logger.info(f"Checkpoint written: {done.path} ({done.bytes / 1e9:.2f} GB, "
                                f"stall {done.stall_s:.3f}s, durable after {done.total_s:.2f}s)")
                    prune_consumed()
            except Exception as e:  # noqa: BLE001 - becomes this rank's vote for the error path
                if pending_err is None:
                    pending_err = e
            boundary.count = float(batch.num_items) if batch is not None else 0.0
            # the periodic save is decided from the agreed step alone and taken only after the
            # vote passed on every rank: a rank that failed in the previous step stops all of
            # them at the vote instead of leaving its peers inside the save's collectives
            save_due = bool(save_every) and training_step % save_every == 0 and training_step != last_save_step
            boundary(save_due=save_due)
            if batch is None:  # unreachable: a local error always stops every rank above
                raise RuntimeError("no batch")
            if save_due:
                st_ = save_checkpoint(blocking=args.no_async_checkpoint, step_now=training_step)
                last_save_step = training_step
                if args.no_async_checkpoint and st_ is not None:
                    prune_consumed()

            if prof_range is not None and training_step == prof_range[0] and prof is None:
                acts = [torch.profiler.ProfilerActivity.CPU]
                if device.type == "cuda":
                    acts.append(torch.profiler.ProfilerActivity.CUDA)
                prof = torch.profiler.profile(activities=acts, record_shapes=True)
                prof.__enter__()

            # ---- compute: K micro-batches, collectives in the last backward, optimizer, schedule
            if inv_static is not None:
                inv = inv_static
            else:
                c = torch.tensor([max(1.0, boundary.count_sum)], dtype=torch.float64).reciprocal_().float()
                inv = c.to(device, non_blocking=True)
            if graphed is not None:
                inv_dev.copy_(inv, non_blocking=True)
                lr_now = optimizer.param_groups[0]["lr"]
                # A failure of this rank's share of the step before the replay: the replay still
                # runs, poisoned (NaN loss scale -> NaN gradients in every captured collective), so
                # the peers' replays complete, every rank's non-finite guard skips the update and
                # the vote stops everyone on this step -- the eager path's poison_and_complete.
                for ph in ("forward", "backward", "optimizer"):
                    try:
                        fault.fire(training_step, ph)
                    except Exception as e:  # noqa: BLE001
                        logger.error(f"Training error at step {training_step} ({ph}, graph mode): {e!r}")
                        pending_err = e
                        inv_dev.fill_(float("nan"))
                        break
                try:
                    if graphed.ready:
                        if ckpt["engine"] is not None:
                            ckpt["engine"].fence()  # the replay's optimizer must follow a pending snapshot
                        loss = graphed.step(batch.inputs, batch.labels)  # optimizer(k-1) + fwd/bwd(k)
                    else:
                        loss = graphed.prime(batch.inputs, batch.labels)  # eager fwd/bwd(k), capture
                    loss = loss.detach().clone()
                except Exception as e:  # noqa: BLE001
                    # capture / replay itself failed: its collectives cannot be completed from here
                    # (they live inside the graph), so this rank leaves like a lost peer
                    raise _FatalStepError(f"HIP graph {'replay' if graphed.ready else 'capture'} failed at "
                                          f"step {training_step}: {e!r}") from e
                if pending_err is None:
                    try:
                        fault.fire(training_step, "post")
                    except Exception as e:  # noqa: BLE001 - after a complete step: nothing to poison
                        logger.error(f"Training error at step {training_step} (post, graph mode): {e!r}")
                        pending_err = e
                phase = "graph"
            tok_all = batch.inputs.to(device, non_blocking=True) if graphed is None else None
            lab_all = batch.labels.to(device, non_blocking=True) if graphed is None else None
            phase = "forward" if graphed is None else "graph"
            if graphed is None:
                loss = None
            try:
                if graphed is not None:
                    raise _GraphDone()
                for k in range(K):
                    reducer.begin_micro(k, K)
                    tok, lab = tok_all[k * B : (k + 1) * B], lab_all[k * B : (k + 1) * B]
                    fault.fire(training_step, "forward")
                    if k == K - 1 and fault.at(training_step, "backward"):
                        reducer.fault_after_buckets = 1
                    lk = model(tok, lab, inv)
                    phase = "backward"
                    lk.backward()
                    loss = lk.detach() if loss is None else loss + lk.detach()
                    phase = "forward"
                phase = "finish"
                reducer.finish()
                phase = "optimizer"
                fault.fire(training_step, "optimizer")
                optimizer.clip_grad_norm_(args.grad_max_norm)
                if ckpt["engine"] is not None:
                    ckpt["engine"].fence()
                lr_now = optimizer.param_groups[0]["lr"]
                phase = "step"
                optimizer.step()
                phase = "schedule"
                lr_scheduler.step()
                phase = "post"
                fault.fire(training_step, "post")
            except _GraphDone:
                pass
            except Exception as e:  # noqa: BLE001
                logger.error(f"Training error at step {training_step} ({phase}): {e!r}")
                pending_err = e
                reducer.fault_after_buckets = 0
                try:
                    _complete_step(phase, reducer, optimizer, lr_scheduler, (K * B, S), emb_dim,
                                   fence=ckpt["engine"].fence if ckpt["engine"] is not None else None)
                except Exception as e2:  # noqa: BLE001
                    raise _FatalStepError(f"could not complete step {training_step} after {e!r}: {e2!r}") from e2
                lr_now = optimizer.param_groups[0]["lr"]
            steps_window += 1

            if pending_err is None and (training_step == 1 or training_step % args.logging_frequency == 0):
                extra = {"lr": f"{lr_now:.3e}"}
                if device.type == "cuda":
                    extra["peak_HBM_GB"] = f"{torch.cuda.max_memory_allocated(device) / 2**30:.1f}"
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
        complete_pending()
        boundary.count = 0.0
        boundary(final=True)  # drains the loss log, last non-finite check, last signals
        if ckpt["engine"] is not None:
            ckpt["engine"].wait()
        log_digest(training_step)
        logger.info("Training completed")
    except _StopTraining as stop:
        e = stop.cause
        exit_type = classify_exception(e)
        try:
            if ckpt["engine"] is not None:
                ckpt["engine"].wait()
        except Exception as we:  # noqa: BLE001
            logger.error(f"previous checkpoint write failed: {we!r}")
        step_now = training_step

        def _save():
            with monitor.blocked():
                st = save_checkpoint(blocking=True, step_now=step_now)
            if st is not None:
                logger.info(f"Checkpoint {st.path}: {st.bytes / 1e9:.2f} GB in {st.total_s:.2f}s "
                            f"(mode {st.mode})")
                log_digest(step_now, " (saved)")
                prune_consumed()

        if exit_type == -1 and not isinstance(e, InjectedFault) and info.is_main:
            logger.error(f"Training error: {e!r}")
        handle_exit(_save, step_now, exit_type, logger, job_id=job_id,
                    sbatch_script=args.sbatch_script, is_main=info.is_main, rank=info.rank)
    except (fdist.PeerFailure, _FatalStepError) as e:
        # a peer vanished (or this rank cannot finish its share of a step): no collective
        # is possible any more. A survivor with complete, replicated state writes the
        # checkpoint alone; then exit non-zero at once (process-group teardown could block
        # on collectives that will never complete).
        logger.error(f"[EXIT HANDLER] Lost a peer rank: {e}")
        step_now = training_step
        if ckpt["engine"] is not None:
            try:  # a save already published by every rank counts; one stuck on the dead peer does not
                ckpt["engine"].poll()
            except Exception:  # noqa: BLE001
                pass
            ok = [h for h in ckpt["engine"].history if not h.error]
            if ok:
                durable.update(step=ok[-1].step, path=ok[-1].path)
        if durable["step"] is not None:
            logger.error(f"[EXIT HANDLER] Last durable checkpoint: {durable['path']} at step {durable['step']} "
                         f"(resume with --checkpoint-id {job_id})")
        else:
            logger.error("[EXIT HANDLER] No durable checkpoint was written by this job")
        complete = isinstance(e, fdist.PeerFailure) and pending_err is None
        if complete and info.distributed and device.type == "cuda" and not _drained(device, 0.5 * info.peer_timeout_s):
            logger.error("[EXIT HANDLER] the last step's collectives never completed; no complete state to save")
            complete = False
        if complete and info.distributed:
            try:
                # graph mode: the last replay's backward has no optimizer step yet (it runs in the
                # next replay). Its gradients are complete (drained above) and the all-reduce mode's
                # optimizer issues no collective, so run it here: the file then records
                # training_step with every one of its updates, as at a clean boundary. (ZeRO-1's
                # optimizer all-gathers would wait on the lost peer; save_solo refuses that mode.)
                if not optimizer.zero1:
                    complete_pending()
                rollback_to_first_bad()
                step_now = training_step
                with monitor.blocked():
                    st = save_solo(step_now)
                if st:
                    logger.error(f"[rank {info.rank}] [EXIT HANDLER] Checkpoint saved at step {step_now}")
            except Exception as se:  # noqa: BLE001
                logger.error(f"[EXIT HANDLER] Checkpoint could not be saved at step {step_now}: {se!r}")
        exit_code = 1
    finally:
        loader.close()
        if metrics_f is not None:
            metrics_f.close()
        monitor.uninstall()
        if ckpt["engine"] is not None and not exit_code:
            ckpt["engine"].preallocated(None)  # never exit while the pinning thread is inside hipHostMalloc
    sys.stdout.flush()
    sys.stderr.flush()
    if exit_code:
        for h in logger.handlers:
            h.flush()
        os._exit(exit_code)
    return 0


def _drained(device: torch.device, timeout_s: float) -> bool:
    """Wait (bounded) until every stream of ``device`` has finished its queued work: a
    collective whose peer died never completes, and a plain device sync would block forever."""
    import threading

    t = threading.Thread(target=torch.cuda.synchronize, args=(device,), daemon=True)
    t.start()
    t.join(timeout_s)
    return not t.is_alive()


def _complete_step(phase: str, reducer, optimizer, lr_scheduler, tokens_shape, dim: int, fence=None) -> None:
    """After a failure at ``phase``, finish this rank's share of the step so the peers'
    collectives complete: unlaunched buckets go out poisoned (NaN), so every rank's
    non-finite guard skips the step's update; then the optimizer/scheduler steps run as
    on the peers. Failures before backward's last bucket poison the whole step; a
    failure after ``optimizer.step()`` was enqueued leaves a valid, complete step.
    ``fence``: the checkpoint engine's snapshot fence — an async periodic snapshot still
    copying the state must finish before this optimizer step writes it (as in the loop)."""
    if phase in ("forward", "backward", "finish", "optimizer"):
        # at "optimizer" the gradients are complete and every bucket went out with valid
        # data: the peers' step is valid, so this rank takes the same valid step
        if phase != "optimizer":
            reducer.poison_and_complete(tokens_shape, dim)
        if fence is not None:
            fence()
        optimizer.step()
        lr_scheduler.step()
    elif phase == "step":
        raise RuntimeError("failure inside optimizer.step(): its collectives may be half issued")
    elif phase == "schedule":
        lr_scheduler.step()


def main(argv=None) -> None:
    args = get_args(argv)
    rc = train(args)
    fdist.destroy()
    sys.exit(rc)


if __name__ == "__main__":
    main()
