#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S pytest_gpu 500 python -m pytest tests -m gpu -x -q || exit 1
$S b_auto 300 python bench.py --steps 10 --warmup 3 || exit 1
FT_DW_TRANSPOSE=none $S b_none 300 python bench.py --steps 10 --warmup 3 || exit 1
FT_DW_TRANSPOSE=all $S b_all 300 python bench.py --steps 10 --warmup 3 || exit 1
$S b_auto2 300 python bench.py --steps 10 --warmup 3 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$S prof4 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 || exit 1
