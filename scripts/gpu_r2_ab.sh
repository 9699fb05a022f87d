#!/bin/bash
# Process-level A/B of env knobs on the GPT-2 presets (alternating rounds).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in 1 2; do
  for v in auto all; do
    for m in gpt2-small gpt2-medium; do
      g=""; [ $m = gpt2-small ] && g="--graph"
      out=$(FT_DW_TRANSPOSE=$v timeout -k 10 180 python3 bench.py --model $m --steps 30 --warmup 5 --no-ckpt $g 2>/dev/null) || exit $?
      echo "round $r FT_DW_TRANSPOSE=$v $m $g: $(echo "$out" | grep -o '"ms_per_step": [0-9.]*')" | tee -a gpurun_out/ab_dw.log
    done
  done
done
