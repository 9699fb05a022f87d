#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S ktest 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_ft_gpu.py tests/test_dp_rccl_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
FT_DEFER_EMB=0 $S bench_nodefer 600 python bench.py || exit 1
$S bench_defer 600 python bench.py || exit 1
FT_DEFER_EMB=0 $S bench_nodefer2 600 python bench.py || exit 1
$S bench_defer2 600 python bench.py || exit 1
