#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S pytest_gpu 500 python -m pytest tests -m gpu -x -q || exit 1
$S b_gpt2m 300 python bench.py --model gpt2-medium --steps 20 --warmup 5 || exit 1
$S b_gpt2s 300 python bench.py --model gpt2-small --steps 20 --warmup 5 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$S prof_gpt2m 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g2m -o run --output-format csv -- python3 bench.py --model gpt2-medium --steps 5 --warmup 3 || exit 1
