#!/bin/bash
# GPT-2 presets under the HIP graph: 128-tile forward GEMMs (FT_GEMM_S) on vs off, alternating rounds.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm_s" > gpurun_out/gemm_s_tests.log 2>&1 || { tail -20 gpurun_out/gemm_s_tests.log; exit 1; }
tail -1 gpurun_out/gemm_s_tests.log
for r in 1 2 3; do
  for cfg in "FT_GEMM_S=1" "FT_GEMM_S=0"; do
    for m in gpt2-small gpt2-medium; do
      ms=$(env $cfg timeout -k 10 200 python bench.py --model $m --graph --steps 50 --warmup 5 --no-ckpt 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['mfu_vs_2.5PF_dense'])") || exit 1
      echo "round $r $m $cfg: $ms (ms/step, mfu)" | tee -a gpurun_out/gpt2_s_ab.log
    done
  done
done
