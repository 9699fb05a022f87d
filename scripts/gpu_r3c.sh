#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S ab_sumsq 600 python -u scripts/ab_step.py --knobs sumsq_end --rounds 4 --steps 8 || exit 1
