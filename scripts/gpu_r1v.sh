#!/bin/bash
# clean (serial optimizer) kernel profile of the current 8B step
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$S prof_v 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --whole-buffer-optimizer || exit 1
