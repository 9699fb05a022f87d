#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S fr_2k 300 python scripts/mem_probe.py --free-run --steps 6 || exit 1
$S fr_2k_t 300 python scripts/mem_probe.py --free-run --throttle --steps 6 || exit 1
$S fr_16k 400 python scripts/mem_probe.py --free-run --steps 4 --seq-len 16384 || exit 1
$S fr_16k_t 400 python scripts/mem_probe.py --free-run --throttle --steps 4 --seq-len 16384 || exit 1
PYTORCH_HIP_ALLOC_CONF=max_split_size_mb:512 $S fr_16k_tm 400 python scripts/mem_probe.py --free-run --throttle --steps 4 --seq-len 16384 || exit 1
