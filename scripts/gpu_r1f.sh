#!/bin/bash
# A/B optimizer scheduling + hipBLASLt TunableOp GEMM selection
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S b_default 300 python bench.py --steps 10 --warmup 3 || exit 1
$S b_whole 300 python bench.py --steps 10 --warmup 3 --whole-buffer-optimizer || exit 1
$S b_serial 300 python bench.py --steps 10 --warmup 3 --no-overlap || exit 1
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results.csv $S b_tune 900 python bench.py --steps 2 --warmup 2 || exit 1
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results.csv $S b_tuned 300 python bench.py --steps 10 --warmup 3 || exit 1
$S b_default2 300 python bench.py --steps 10 --warmup 3 || exit 1
ls -la gpurun_out/
