#!/bin/bash
# fused FFN (tiled SwiGLU with transposed outputs): numerics, then 8B A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S ffn_tests 400 python -m pytest tests/test_kernels_gpu.py -x -q -k "swiglu or feed_forward or tiny_model or weight_grad" || exit 1
$S b_fused 300 python bench.py --steps 10 --warmup 3 || exit 1
FT_FUSED_FFN=0 $S b_unfused 300 python bench.py --steps 10 --warmup 3 || exit 1
$S b_fused2 300 python bench.py --steps 10 --warmup 3 || exit 1
FT_FUSED_FFN=0 $S b_unfused2 300 python bench.py --steps 10 --warmup 3 || exit 1
