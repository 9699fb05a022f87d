#!/bin/bash
# kernel trace of the current 8B step (pipelined optimizer, dW side stream)
export TMPDIR=/tmp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 4 --warmup 2 > gpurun_out/prof.log 2>&1 || exit 1
find gpurun_out/prof -name "*.csv" | head
