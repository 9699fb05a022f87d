#!/bin/bash
# GPT-2-small / -medium MFU at 1 / 8 / 16 sequences per GPU under the whole-step HIP graph (README row).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for m in gpt2-small gpt2-medium; do
  for b in 1 8 16; do
    timeout -k 10 200 python bench.py --model $m --graph --batch-size $b --steps 30 --warmup 5 --no-ckpt > gpurun_out/b_${m}_$b.log 2>&1 || { tail -5 gpurun_out/b_${m}_$b.log; exit 1; }
    echo "$m bs $b: $(tail -1 gpurun_out/b_${m}_$b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/step", round(d["value"]), "tok/s", "mfu", d.get("mfu_vs_2.5PF_dense"))')"
  done
done
