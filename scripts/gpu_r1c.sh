#!/bin/bash
# Full GPU check: all gpu tests, 8B bench, rocprofv3 kernel stats of the 8B bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S pytest_gpu 500 python -m pytest tests -m gpu -x -q || exit 1
$S bench_8b 600 python bench.py --steps 10 --warmup 3 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$S prof_8b 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 || exit 1
