#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S ktest 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "swiglu or feed_forward" || exit 1
FT_KERNELS_SO=abso/_kernels_base.so $S kbw_old 300 python -u scripts/kernel_bw_bench.py || exit 1
$S kbw_new 300 python -u scripts/kernel_bw_bench.py || exit 1
