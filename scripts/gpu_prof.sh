#!/bin/bash
# rocprofv3 kernel trace + stats of a short Llama-3-8B bench
export TMPDIR=/tmp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 "$@" > gpurun_out/prof.log 2>&1
rc=$?
echo "rc=$rc"; tail -3 gpurun_out/prof.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
