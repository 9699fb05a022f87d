#!/bin/bash
# Round 6, session E: GPT-2 graph step A/B (round-5 tree vs HEAD vs HEAD with FT_W4_SMALL=0), w4
# product microbenches in both trees (8B), rocprof kernel stats of the GPT-2-small graph step.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
j() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('sclk_mhz_p50'), d.get('power_w_p50'))"; }
for m in gpt2-small gpt2-medium; do for r in 1 2; do for v in r5 head head_w4small0 head_qkvrope; do
  if [ $v = r5 ]; then cd $R/abtree_r5; else cd $R; fi
  if [ $v = head_w4small0 ]; then export FT_W4_SMALL=0; else unset FT_W4_SMALL; fi
  if [ $v = head_qkvrope ]; then export FT_QKV_ROPE_MIN_K=768; else unset FT_QKV_ROPE_MIN_K; fi
  timeout -k 10 300 python -u bench.py --model $m --vocab-size 50304 --graph --steps 50 --warmup 5 --no-ckpt > $R/gpurun_out/r6e_${m}_${v}_$r.log 2>&1 || exit 1
  echo "$m $v $r $(j $R/gpurun_out/r6e_${m}_${v}_$r.log)"
done; done; done
unset FT_W4_SMALL FT_QKV_ROPE_MIN_K
for v in r5 head; do
  if [ $v = r5 ]; then cd $R/abtree_r5; else cd $R; fi
  timeout -k 10 300 python -u scripts/gemm_w4t_bench.py > $R/gpurun_out/r6e_w4t_$v.log 2>&1 || exit 1
  timeout -k 10 300 python -u scripts/w4_split_bench.py > $R/gpurun_out/r6e_split_$v.log 2>&1 || exit 1
done
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6e_prof_gpt2s -o run --output-format csv -- \
  python3 bench.py --model gpt2-small --vocab-size 50304 --graph --steps 20 --warmup 3 --no-ckpt > gpurun_out/r6e_prof_gpt2s.log 2>&1 || exit 1
python scripts/prof_summary.py $(ls gpurun_out/r6e_prof_gpt2s/*/run_kernel_stats.csv gpurun_out/r6e_prof_gpt2s/run_kernel_stats.csv 2>/dev/null | head -1) "GPT-2-small vocab 50304 --graph, HEAD" 23 > gpurun_out/r6e_gpt2s_kernel_stats.md
head -30 gpurun_out/r6e_gpt2s_kernel_stats.md
