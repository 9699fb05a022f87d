"""Command-line surface.

The 16 reference flags are kept byte-for-byte (names, types, defaults, help):
reference ``utils.py:112-203`` (table in SURVEY.md §2.6). Everything after the
``# --- additive flags ---`` marker is new and defaults to the reference's
behaviour.
"""
from __future__ import annotations

import argparse
import os

import torch

PRECISION_STR_TO_DTYPE = {
    "fp16": torch.float16,
    "bf16": torch.bfloat16,
    "fp32": torch.float32,
    "fp64": torch.float64,
}


def workdir() -> str:
    """``$WORKDIR`` (reference ``utils.py:11``)."""
    return os.getenv("WORKDIR", "")


def jobid() -> str | None:
    """``$SLURM_JOB_ID`` (reference ``utils.py:12``; read at call time, not import time)."""
    return os.environ.get("SLURM_JOB_ID")


def build_parser() -> argparse.ArgumentParser:
    wd = workdir()
    parser = argparse.ArgumentParser()
    parser.add_argument(
        "--dataset",
        type=str,
        default="/capstor/store/cscs/ethz/large-sc/datasets/train_data.parquet",
        help="Path to a parquet file containing a 'text' column with documents (`str`)",
    )
    parser.add_argument(
        "--checkpoint-path",
        type=str,
        default=f"{wd}/checkpoints",
        help="Path to a checkpoint file to save the model and optimizer state dicts",
    )
    parser.add_argument(
        "--checkpoint-id",
        type=str,
        default="",
        help="Path to a checkpoint file to save the model and optimizer state dicts",
    )
    parser.add_argument(
        "--tokenizer-name-or-path",
        type=str,
        default="unsloth/Mistral-Nemo-Base-2407-bnb-4bit",
        help="A path to a directory containing vocabulary files required by the tokenizer or the model id of a predefined tokenizer hosted inside a model repo on the Hugging Face Hub.",
    )
    parser.add_argument("--sequence-length", type=int, default=4096)
    parser.add_argument("--batch-size", type=int, default=1)
    parser.add_argument(
        "--fused-optimizer",
        action="store_true",
        help="Set to fuse the optimizer for increased performance or not",
    )
    parser.add_argument("--learning-rate", type=float, default=1e-5)
    parser.add_argument("--lr-warmup-steps", type=int, default=10)
    parser.add_argument("--training-steps", type=int, default=1000)
    parser.add_argument(
        "--logging-frequency", type=int, default=5, help="Log every `--logging-frequency` steps"
    )
    parser.add_argument("--grad-max-norm", type=float, default=1)
    parser.add_argument(
        "--model-dtype",
        type=str,
        default="bf16",
        help="Model dtype for parameters, gradients and optimizer states. Default: bf16",
    )
    parser.add_argument(
        "--compile", action="store_true", help="Set to compile the model with `torch.compile`"
    )
    parser.add_argument(
        "--raise-error",
        action="store_true",
        help="Set to raise an error in the training loop at the error_step parameter",
    )
    parser.add_argument(
        "--error-step",
        type=int,
        default=100,
        help="Step at which to raise an error if --raise-error is set",
    )
    # --- additive flags (not in the reference; defaults keep its behaviour) ---
    parser.add_argument(
        "--model",
        type=str,
        default="llama3-8b",
        help="Architecture preset: llama3-8b (reference train.py:43-53), gpt2-small, gpt2-medium, tiny",
    )
    parser.add_argument(
        "--vocab-size",
        type=int,
        default=0,
        help="Override the vocabulary size (0: tokenizer's, or 131072 with --synthetic-data)",
    )
    parser.add_argument(
        "--synthetic-data",
        action="store_true",
        help="Deterministic synthetic token stream instead of parquet+tokenizer (offline boxes)",
    )
    parser.add_argument(
        "--iterable-dataset",
        action="store_true",
        help="Use the packing IterableParquetDataset (resumable mid-shard) instead of ParquetDataset",
    )
    parser.add_argument("--seed", type=int, default=1234, help="RNG seed for init and data")
    parser.add_argument(
        "--state-digest",
        action="store_true",
        help="At 'Training completed', log bit-level digests of the parameters, AdamW moments and "
        "data-loader position (resume-equivalence checks without a second checkpoint on disk)",
    )
    parser.add_argument(
        "--device", type=str, default="cuda", choices=["cuda", "cpu"], help="Run on GPU (default) or CPU"
    )
    parser.add_argument(
        "--save-every",
        type=int,
        default=-1,
        help="Periodic asynchronous checkpoint every N steps (0 disables; default: 200 under data "
        "parallelism, so a lost rank costs at most that many steps, else 0)",
    )
    parser.add_argument(
        "--no-async-checkpoint",
        action="store_true",
        help="Block the training loop until each periodic checkpoint is durable",
    )
    parser.add_argument(
        "--checkpoint-mode",
        type=str,
        default="auto",
        choices=["auto", "hbm", "host"],
        help="Snapshot path: hbm = D2D copy into reserved HBM then background D2H; host = D2H "
        "straight into pinned host memory; auto = hbm when free HBM allows",
    )
    parser.add_argument(
        "--checkpoint-alt-path",
        type=str,
        default="",
        help="A second checkpoint directory (another filesystem): a job that resumed from a file in one "
        "of the two directories writes its own checkpoints to the other, so the file it resumed from "
        "stays intact until its own is durable (a disk with room for ONE checkpoint, e.g. the 48 GB 8B "
        "file on 79 GB). --checkpoint-id is looked up in both",
    )
    parser.add_argument(
        "--prune-consumed",
        action="store_true",
        help="Delete the checkpoint this job resumed from once this job's own checkpoint is durable "
        "(periodic or exit save): the chain keeps at least one complete checkpoint at every moment",
    )
    parser.add_argument(
        "--no-checkpoint-prealloc",
        action="store_true",
        help="Pin the checkpoint host buffers at the first save instead of in a background thread at startup",
    )
    parser.add_argument(
        "--checkpoint-writer-threads", type=int, default=8, help="Parallel pwrite threads of the checkpoint writer"
    )
    parser.add_argument(
        "--prefetch", type=int, default=2, help="Batches prepared ahead by the data-loader thread (0: inline)"
    )
    parser.add_argument(
        "--optimizer-state-dtype",
        type=str,
        default="",
        help="AdamW moment dtype (bf16/fp16/fp32); default = --model-dtype like the reference (fp32 for fp16 models: fp16 moments underflow)",
    )
    parser.add_argument(
        "--dp-bucket-mb",
        type=float,
        default=None,
        help="Gradient bucket size in MiB: the all-reduce / reduce-scatter unit under data parallelism "
             "(default 256) and the optimizer's launch / gating unit on one GPU (default 64)",
    )
    parser.add_argument(
        "--dp-mode",
        type=str,
        default="",
        choices=["", "allreduce", "zero1"],
        help="Data-parallel gradient mode (default zero1: reduce-scatter + sharded AdamW + all-gather)",
    )
    parser.add_argument(
        "--dp-reduce-dtype",
        type=str,
        default="native",
        choices=["native", "fp32"],
        help="Data-parallel gradient reduction dtype: native (the gradient dtype, bf16 by default; the "
        "error bound is in docs/PERFORMANCE.md) or fp32 (reduce an fp32 copy of each bucket: 2x the "
        "bytes on the links, one rounding)",
    )
    parser.add_argument(
        "--grad-accum",
        type=int,
        default=1,
        help="Gradient accumulation: micro-batches of --batch-size per optimizer step (collectives only "
        "in the last micro-batch's backward)",
    )
    parser.add_argument(
        "--hip-graph",
        action="store_true",
        help="Replay each step (optimizer of the previous step + forward/backward) as one HIP graph; "
        "1 GPU, no gradient accumulation. For launch-bound small models (gpt2-small: -18%% step time)",
    )
    parser.add_argument(
        "--peer-timeout",
        type=float,
        default=60.0,
        help="Seconds a rank waits at the per-step vote for a silent peer before declaring it lost "
        "(a dead peer is detected at once); well under Slurm's 120 s USR1 lead",
    )
    parser.add_argument(
        "--flash-bwd",
        type=str,
        default="deterministic",
        choices=["deterministic", "atomic"],
        help="Flash-attention backward: atomic-free dQ kernel (bit-reproducible, default) or fp32 atomics",
    )
    parser.add_argument(
        "--activation-checkpointing",
        type=int,
        default=0,
        help="Recompute this many transformer blocks (from the first; -1 = all) in backward instead of "
        "storing their activations (long sequences / larger batches per GPU)",
    )
    parser.add_argument(
        "--recompute-attention",
        action="store_true",
        help="With --activation-checkpointing: also re-run the flash-attention forward in backward "
        "(default keeps each recomputed block's attention output: one T x Hq x D tensor per block)",
    )
    parser.add_argument(
        "--profile-steps",
        type=str,
        default="",
        help="torch.profiler window 'START:STOP' (steps); Chrome trace written to --profile-dir",
    )
    parser.add_argument("--profile-dir", type=str, default="profiles/torch", help="Output dir for --profile-steps")
    parser.add_argument(
        "--metrics-file", type=str, default="", help="Append per-step JSON metrics to this file"
    )
    parser.add_argument(
        "--sbatch-script",
        type=str,
        default="",
        help="Job script resubmitted on SIGUSR1 (default: $WORKDIR/train.sh)",
    )
    return parser


def get_args(argv=None) -> argparse.Namespace:
    """Parse flags (reference ``utils.py:112-203``)."""
    return build_parser().parse_args(argv)
