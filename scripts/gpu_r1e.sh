#!/bin/bash
# A/B: AdamW grid caps under overlap; 1-rank RCCL zero1/allreduce paths; O_DIRECT checkpoint save
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S pytest_gpu 500 python -m pytest tests -m gpu -x -q || exit 1
$S b_default 300 python bench.py --steps 10 --warmup 3 || exit 1
FT_ADAMW_BLOCKS=256 $S b_blk256 300 python bench.py --steps 10 --warmup 3 || exit 1
FT_ADAMW_BLOCKS=512 $S b_blk512 300 python bench.py --steps 10 --warmup 3 || exit 1
$S b_serial 300 python bench.py --steps 10 --warmup 3 --no-overlap || exit 1
FT_FORCE_DIST=1 $S b_zero1 300 python bench.py --steps 10 --warmup 3 --dp-mode zero1 || exit 1
FT_FORCE_DIST=1 $S b_allreduce 300 python bench.py --steps 10 --warmup 3 --dp-mode allreduce || exit 1
mkdir -p /tmp/ftck
$S b_ckpt 400 python bench.py --steps 3 --warmup 2 --ckpt-dir /tmp/ftck || exit 1
