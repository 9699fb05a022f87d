#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S ktest 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "adamw or pipelined" || exit 1
for v in 0 1 2 0 1 2; do FT_ADAMW_VARIANT=$v $S bw_v$v 300 python -u scripts/bw_bench.py || exit 1; grep "adamw blocks=     0" gpurun_out/bw_v$v.log >> gpurun_out/bw_var.txt; echo "v$v" >> gpurun_out/bw_var.txt; done
