#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S ftgpu 600 python -u -m pytest tests/test_ft_gpu.py -m gpu -x -v --timeout 400 --timeout-method thread || exit 1
