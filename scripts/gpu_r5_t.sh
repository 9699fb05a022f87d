#!/bin/bash
# Round 5, session T: GPT-2 QKV projection with the RoPE epilogue (gate lowered) vs w4 + RoPE kernel, --graph bench alternated.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for v in off on off on; do
  for m in gpt2-small gpt2-medium; do
    timeout -k 10 300 python -u -c "
import sys, runpy
from fault_tolerant_llm_training_amd.ops import attention as A
A._QKV_ROPE_MIN_K = 0 if '$v' == 'on' else A._QKV_ROPE_MIN_K
sys.argv = ['bench.py', '--model', '$m', '--vocab-size', '50304', '--graph', '--steps', '30', '--warmup', '5', '--no-ckpt']
runpy.run_path('bench.py', run_name='__main__')
" > gpurun_out/r5t_${m}_$v.log 2>&1 || exit 1
    echo "$m qkvrope=$v $(tail -1 gpurun_out/r5t_${m}_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("sclk_mhz_p50"))')" | tee -a gpurun_out/r5t_summary.log
  done
done
