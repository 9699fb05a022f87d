#!/bin/bash
# Round 6, session AU: where the GPT-2-small graph step dies with GPU_MAX_HW_QUEUES=2 (faulthandler).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
GPU_MAX_HW_QUEUES=2 timeout -k 10 200 python -X faulthandler -u bench.py --model gpt2-small --vocab-size 50304 --graph --steps 10 --warmup 3 --no-ckpt > gpurun_out/r6au.log 2>&1
echo "rc=$?"; grep -v amdgpu.ids gpurun_out/r6au.log | tail -40
