#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S gputests 600 python -u -m pytest tests/test_flash_attn_gpu.py tests/test_kernels_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
$S ab_dqs 600 python -u scripts/ab_step.py --knobs dqs --rounds 4 --steps 8 || exit 1
