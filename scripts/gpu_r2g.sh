#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S ab_prio 600 python -u scripts/ab_step.py --knobs prio,dw --rounds 3 --steps 8 || exit 1
