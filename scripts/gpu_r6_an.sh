#!/bin/bash
# Round 6, session AN: same box, alternating: the tree at the start of this session (46f5b90, built in
# abtree_r5/) vs HEAD -- 8B bench step and GPT-2-small / -medium graph steps.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for t in old new old new; do
  if [ $t = old ]; then d=abtree_r5; else d=.; fi
  (cd $d && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-ckpt) > gpurun_out/r6an_b.json 2>gpurun_out/r6an_b.err || { tail -3 gpurun_out/r6an_b.err; exit 1; }
  echo "8b $t $(python3 -c "import json;d=json.loads(open('gpurun_out/r6an_b.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d.get('sclk_mhz_p50'), d.get('power_w_p50'))")" | tee -a gpurun_out/r6an.log
done
for m in gpt2-small gpt2-medium; do
  for t in old new old new; do
    if [ $t = old ]; then d=abtree_r5; else d=.; fi
    (cd $d && timeout -k 10 300 python -u bench.py --model $m --vocab-size 50304 --graph --steps 50 --warmup 5 --no-ckpt) > gpurun_out/r6an_b.json 2>gpurun_out/r6an_b.err || { tail -3 gpurun_out/r6an_b.err; exit 1; }
    echo "$m $t $(python3 -c "import json;d=json.loads(open('gpurun_out/r6an_b.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d.get('sclk_mhz_p50'))")" | tee -a gpurun_out/r6an.log
  done
done
