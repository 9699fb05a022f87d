#!/bin/bash
export TMPDIR=/tmp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fprof -o run --output-format csv -- python3 scripts/flash_bench.py > gpurun_out/fprof.log 2>&1 || exit 1
