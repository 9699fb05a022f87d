#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S pytest_kernels 400 python -m pytest tests/test_kernels_gpu.py -x -q || exit 1
$S bench_small 300 python bench.py --model gpt2-small --steps 10 --warmup 3 || exit 1
$S bench_8b 600 python bench.py --steps 10 --warmup 3 || exit 1
