#!/bin/bash
# norm dW fold on the dW side stream: numerics + step A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S nf_test 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_dp_rccl_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
$S nf_bench 300 python bench.py || exit 1
FT_NORM_FOLD_SIDE=0 $S nf_bench_old 300 python bench.py || exit 1
$S nf_bench2 300 python bench.py || exit 1
FT_NORM_FOLD_SIDE=0 $S nf_bench_old2 300 python bench.py || exit 1
$S nf_bench3 300 python bench.py || exit 1
FT_NORM_FOLD_SIDE=0 $S nf_bench_old3 300 python bench.py || exit 1
for f in nf_bench nf_bench_old nf_bench2 nf_bench_old2 nf_bench3 nf_bench_old3; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log)"; done
