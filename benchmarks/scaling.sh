#!/bin/bash
# DP scaling curve on one node: bench.py at N = 1, 2, 4, 8 MI355X (one process per GPU, RCCL/xGMI).
# Prints bench.py's JSON line for every N (value = whole-job tokens/s), then one summary line with
# tokens/s per GPU and weak-scaling efficiency vs N=1. N larger than the visible GPU count is skipped.
# Usage: benchmarks/scaling.sh [steps] [warmup] [extra bench args]
STEPS=${1:-10}; WARM=${2:-3}; shift 2 2>/dev/null
export HSA_ENABLE_IPC_MODE_LEGACY=0
NGPU=$(python -c "import torch; print(torch.cuda.device_count())")
OUT=$(mktemp)
for N in 1 2 4 8; do
  [ "$N" -gt "$NGPU" ] && { echo "{\"skipped\": $N, \"reason\": \"only $NGPU GPUs visible\"}"; continue; }
  if [ "$N" = 1 ]; then
    python bench.py --gpus 1 --steps $STEPS --warmup $WARM --no-ckpt "$@" | tee -a "$OUT"
  else
    python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
      --master-port $((29600 + N)) bench.py --gpus $N --steps $STEPS --warmup $WARM --no-ckpt "$@" | tee -a "$OUT"
  fi
done
python - "$OUT" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
base = next((r["tokens_per_s_per_gpu"] for r in rows if r.get("n_gpus") == 1), None)
print(json.dumps({"scaling_summary": [
    {"n_gpus": r["n_gpus"], "tok_s_per_gpu": r["tokens_per_s_per_gpu"], "ms_per_step": r["ms_per_step"],
     "exposed_comm_ms_per_step": r.get("exposed_comm_ms_per_step"),
     "weak_scaling_efficiency": round(r["tokens_per_s_per_gpu"] / base, 3) if base else None} for r in rows]}))
PY
rm -f "$OUT"
