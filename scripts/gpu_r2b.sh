#!/bin/bash
# Tune the 8B step's GEMM solutions (TunableOp) and A/B them in one process; copy the table out.
export TMPDIR=/tmp
mkdir -p gpurun_out tuning
S=scripts/gpu_check.sh
$S tune 1000 python -u scripts/tune_gemms.py --out gpurun_out/gemm_gfx950.csv || exit 1
