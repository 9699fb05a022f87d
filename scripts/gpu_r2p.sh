#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S ktest 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
$S kbw 300 python -u scripts/kernel_bw_bench.py || exit 1
