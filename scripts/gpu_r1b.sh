#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S pytest_flash 300 python -m pytest tests/test_flash_attn_gpu.py -x -q || exit 1
$S pytest_kernels 300 python -m pytest tests/test_kernels_gpu.py -x -q || exit 1
$S bench_8b 600 python bench.py --steps 10 --warmup 3 || exit 1
