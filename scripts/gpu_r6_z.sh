#!/bin/bash
# Round 6, session Z: kernel stats of the fp32 GPT-2-medium step with the GEMMs on gemm_f32 (FT_F32_MFMA=1)
# and on hipBLASLt (0).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for v in 1 0; do
  rm -rf gpurun_out/r6z_prof$v
  FT_F32_MFMA=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6z_prof$v -o run --output-format csv -- python3 scripts/ab_step.py --model gpt2-medium --vocab-size 50304 --dtype fp32 --knobs "" --rounds 1 --steps 5 --warmup 2 > gpurun_out/r6z_prof$v.log 2>&1 || exit 1
  python scripts/prof_summary.py $(find gpurun_out/r6z_prof$v -name "run_kernel_stats.csv" | head -1) "fp32 GPT-2-medium step (vocab 50304), FT_F32_MFMA=$v, 7 steps incl. warmup" 7 > gpurun_out/r6z_gpt2m_fp32_mfma$v.md
  head -24 gpurun_out/r6z_gpt2m_fp32_mfma$v.md
  rm -rf gpurun_out/r6z_prof$v
done
