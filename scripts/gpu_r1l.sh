#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S b_def 300 python bench.py --steps 10 --warmup 3 || exit 1
FT_COMPUTE_PRIORITY=1 $S b_prio 300 python bench.py --steps 10 --warmup 3 || exit 1
FT_COMPUTE_PRIORITY=1 FT_ADAMW_BLOCKS=65535 $S b_prio_short 300 python bench.py --steps 10 --warmup 3 || exit 1
FT_ADAMW_BLOCKS=65535 $S b_short 300 python bench.py --steps 10 --warmup 3 || exit 1
$S b_whole 300 python bench.py --steps 10 --warmup 3 --whole-buffer-optimizer || exit 1
$S b_def2 300 python bench.py --steps 10 --warmup 3 || exit 1
