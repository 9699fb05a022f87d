#!/bin/bash
# DP scaling curve on one node: bench.py at N = 1, 2, 4, 8 MI355X (one process per GPU, RCCL/xGMI).
# Prints one JSON line per N (value = whole-job tokens/s). Usage: benchmarks/scaling.sh [steps] [warmup] [extra bench args]
STEPS=${1:-10}; WARM=${2:-3}; shift 2 2>/dev/null
export HSA_ENABLE_IPC_MODE_LEGACY=0
for N in 1 2 4 8; do
  if [ "$N" = 1 ]; then
    python bench.py --gpus 1 --steps $STEPS --warmup $WARM "$@"
  else
    python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
      --master-port $((29600 + N)) bench.py --gpus $N --steps $STEPS --warmup $WARM "$@"
  fi
done
