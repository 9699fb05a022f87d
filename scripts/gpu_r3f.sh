#!/bin/bash
# caching-allocator A/B on the long-context (32k, recompute) and the 2k 8B step
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S al_32k_def 500 python bench.py --seq-len 32768 --steps 3 --warmup 2 --activation-checkpointing -1 || exit 1
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True $S al_32k_exp 500 python bench.py --seq-len 32768 --steps 3 --warmup 2 --activation-checkpointing -1 || exit 1
$S al_2k_def 300 python bench.py || exit 1
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True $S al_2k_exp 300 python bench.py || exit 1
$S al_16k_def 400 python bench.py --seq-len 16384 --steps 3 --warmup 2 || exit 1
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True $S al_16k_exp 400 python bench.py --seq-len 16384 --steps 3 --warmup 2 || exit 1
