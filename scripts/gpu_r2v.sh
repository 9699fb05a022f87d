#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S flashtest 600 python -u -m pytest tests/test_flash_attn_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
$S fb_new 300 python -u scripts/flash_bench.py || exit 1
$S fb_new2 300 python -u scripts/flash_bench.py || exit 1
