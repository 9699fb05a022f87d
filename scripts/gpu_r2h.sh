#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S rccl1 600 python -u -m pytest tests/test_dp_rccl_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
