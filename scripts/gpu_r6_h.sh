#!/bin/bash
# Round 6, session H: the graph-mode RCCL watchdog abort (hipErrorCapturedEvent) -- repeated runs
# with and without TORCH_NCCL_RETHROW_CUDA_ERRORS=0 (dist.graph_capture_env sets it under --compile).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 FT_FORCE_DIST=1 HSA_ENABLE_IPC_MODE_LEGACY=0 SLURM_JOB_ID=900
A="--device cuda --model tiny --synthetic-data --vocab-size 1024 --sequence-length 256 --batch-size 2 --learning-rate 1e-3 --lr-warmup-steps 3 --logging-frequency 5 --training-steps 40 --compile"
n=0
for env in "TORCH_NCCL_RETHROW_CUDA_ERRORS=1" "TORCH_NCCL_RETHROW_CUDA_ERRORS=0"; do for mode in allreduce zero1; do for r in 1 2 3; do
  n=$((n+1)); rm -rf /tmp/ckh; export MASTER_PORT=$((29700+n))
  env $env timeout -k 10 200 python -u train.py $A --dp-mode $mode --checkpoint-path /tmp/ckh > gpurun_out/r6h_$n.log 2>&1
  rc=$?; echo "== $env $mode run $r rc=$rc completed=$(grep -c 'Training completed' gpurun_out/r6h_$n.log) watchdog_err=$(grep -c 'watchdog thread terminated' gpurun_out/r6h_$n.log)"
done; done; done
