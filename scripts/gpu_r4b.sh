#!/bin/bash
# split-row norm backward: numerics, bandwidth A/B, step A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S nb_test 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "norm" --timeout 120 --timeout-method thread || exit 1
$S nb_kbw 200 python scripts/kernel_bw_bench.py || exit 1
$S nb_bench 300 python bench.py || exit 1
FT_NORM_BWD_SPLIT=0 $S nb_bench_old 300 python bench.py || exit 1
$S nb_bench2 300 python bench.py || exit 1
FT_NORM_BWD_SPLIT=0 $S nb_bench_old2 300 python bench.py || exit 1
