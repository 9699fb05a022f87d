#!/bin/bash
# Round 6, session D: same-box A/B of the round-5 tree (abtree_r5, its own kernels) vs HEAD on the
# 8B bench and the GPT-2 graph benches; GPT-2 product probe.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
df -h / /tmp /dev/shm 2>&1 | tee gpurun_out/r6d_df.log; free -g | tee -a gpurun_out/r6d_df.log
timeout -k 10 300 python -u scripts/gpt2_gemm_probe.py > gpurun_out/r6d_gpt2_probe_small.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/gpt2_gemm_probe.py 1024 2816 3072 > gpurun_out/r6d_gpt2_probe_medium.log 2>&1 || exit 1
cut -c1-120 gpurun_out/r6d_gpt2_probe_small.log gpurun_out/r6d_gpt2_probe_medium.log
j() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('sclk_mhz_p50'), d.get('power_w_p50'))"; }
for r in 1 2 3; do for v in r5 head; do
  if [ $v = r5 ]; then cd $R/abtree_r5; else cd $R; fi
  timeout -k 10 300 python -u bench.py --steps 15 --warmup 4 --no-ckpt > $R/gpurun_out/r6d_8b_${v}_$r.log 2>&1 || exit 1
  echo "8b $v $r $(j $R/gpurun_out/r6d_8b_${v}_$r.log)"
done; done
cd $R
for m in gpt2-small gpt2-medium; do for r in 1 2; do for v in r5 head; do
  if [ $v = r5 ]; then cd $R/abtree_r5; else cd $R; fi
  timeout -k 10 300 python -u bench.py --model $m --vocab-size 50304 --graph --steps 50 --warmup 5 --no-ckpt > $R/gpurun_out/r6d_${m}_${v}_$r.log 2>&1 || exit 1
  echo "$m $v $r $(j $R/gpurun_out/r6d_${m}_${v}_$r.log)"
done; done; done
