#!/bin/bash
# GPT-2 presets under the HIP graph: w4 forward GEMMs / QKV+RoPE epilogue on vs off (bench.py, env knobs),
# two alternating rounds.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in 1 2; do
  for cfg in "FT_QKV_ROPE=1 FT_W4_FWD=1" "FT_QKV_ROPE=0 FT_W4_FWD=1" "FT_QKV_ROPE=0 FT_W4_FWD=0"; do
    for m in gpt2-small gpt2-medium; do
      ms=$(env $cfg timeout -k 10 200 python bench.py --model $m --graph --steps 50 --warmup 5 --no-ckpt 2>/dev/null | tail -1 | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])") || exit 1
      echo "round $r $m $cfg: $ms ms/step" | tee -a gpurun_out/gpt2_w4_ab.log
    done
  done
done
