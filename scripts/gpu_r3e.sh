#!/bin/bash
# kernel profile of the seq-32k activation-checkpointed 8B step
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/prof32k; mkdir -p gpurun_out/prof32k
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof32k -o run --output-format csv -- python3 bench.py --seq-len 32768 --steps 2 --warmup 1 --activation-checkpointing -1 > gpurun_out/prof32k.log 2>&1 || exit 1
