#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S kbw 300 python -u scripts/kernel_bw_bench.py || exit 1
