#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S pytest_gpu 500 python -m pytest tests -m gpu -x -q || exit 1
$S flash_bench 300 python scripts/flash_bench.py || exit 1
$S b_def 300 python bench.py --steps 10 --warmup 3 || exit 1
