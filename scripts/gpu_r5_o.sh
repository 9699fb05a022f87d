#!/bin/bash
# Round 5, session O: AdamW serial-vs-overlapped A/B on the 8B step; GPT-2 routing (short-K w4) bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/ab_step.py --knobs adamw_serial --rounds 3 > gpurun_out/r5o_ab_adamw_serial.log 2>&1 || exit 1
grep best gpurun_out/r5o_ab_adamw_serial.log
for m in gpt2-small gpt2-medium; do
  timeout -k 10 300 python -u bench.py --model $m --vocab-size 50304 --graph --steps 30 --warmup 5 --no-ckpt > gpurun_out/r5o_$m.log 2>&1 || exit 1
  tail -1 gpurun_out/r5o_$m.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["model"], d["ms_per_step"], d["mfu_vs_2.5PF_dense"], d.get("sclk_mhz_p50"))'
done
