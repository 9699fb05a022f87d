#!/bin/bash
# Numerics of the changed kernels (norm bwd, NT optimizer pass), NT A/B, dW-stream A/B.
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S gputests 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
FT_STREAM_NT=0 $S bw_plain 300 python -u scripts/bw_bench.py || exit 1
FT_STREAM_NT=1 $S bw_nt 300 python -u scripts/bw_bench.py || exit 1
$S ab_dw 600 python -u scripts/ab_step.py --knobs dw --rounds 3 --steps 8 || exit 1
