#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S b_def 300 python bench.py --steps 10 --warmup 3 || exit 1
$S b_whole 300 python bench.py --steps 10 --warmup 3 --whole-buffer-optimizer || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$S prof_whole 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_whole -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --whole-buffer-optimizer || exit 1
