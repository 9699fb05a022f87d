#!/bin/bash
# round-end style verification of the current tree: GPU tests, smoke, bench, kernel profile
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S gputests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
$S smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
$S bench 600 python bench.py || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof; mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 4 --warmup 2 > gpurun_out/prof.log 2>&1 || exit 1
