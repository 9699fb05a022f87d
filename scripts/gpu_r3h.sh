#!/bin/bash
# caching-allocator split limit A/B: long-context fragmentation and the 2k step
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
PYTORCH_HIP_ALLOC_CONF=max_split_size_mb:512 $S ms_32k_512 500 python bench.py --seq-len 32768 --steps 3 --warmup 2 --activation-checkpointing -1 || exit 1
PYTORCH_HIP_ALLOC_CONF=max_split_size_mb:128 $S ms_32k_128 500 python bench.py --seq-len 32768 --steps 3 --warmup 2 --activation-checkpointing -1 || exit 1
PYTORCH_HIP_ALLOC_CONF=max_split_size_mb:512 $S ms_16k_512 400 python bench.py --seq-len 16384 --steps 3 --warmup 2 || exit 1
$S ms_2k_def 300 python bench.py || exit 1
PYTORCH_HIP_ALLOC_CONF=max_split_size_mb:512 $S ms_2k_512 300 python bench.py || exit 1
$S ms_2k_def2 300 python bench.py || exit 1
PYTORCH_HIP_ALLOC_CONF=max_split_size_mb:512 $S ms_2k_5122 300 python bench.py || exit 1
