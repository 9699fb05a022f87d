#!/bin/bash
# pipelined optimizer: GPU tests, smoke, A/B bench overlap vs serial, kernel profile
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S pytest_gpu 500 python -m pytest tests -m gpu -x -q || exit 1
$S smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
$S bench_overlap 600 python bench.py --steps 10 --warmup 3 || exit 1
$S bench_serial 600 python bench.py --steps 10 --warmup 3 --no-overlap || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$S prof_overlap 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 || exit 1
