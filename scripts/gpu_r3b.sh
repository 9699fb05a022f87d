#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S b_default 600 python bench.py || exit 1
$S b_nooverlap 600 python bench.py --no-overlap || exit 1
$S b_whole 600 python bench.py --whole-buffer-optimizer || exit 1
$S b_default2 600 python bench.py || exit 1
$S b_nooverlap2 600 python bench.py --no-overlap || exit 1
$S b_whole2 600 python bench.py --whole-buffer-optimizer || exit 1
