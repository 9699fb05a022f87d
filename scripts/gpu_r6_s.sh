#!/bin/bash
# Round 6, session S: fp32 GEMM -- staggered start of a CU's second workgroup (s_sleep 48 / 96 x 64
# cycles) vs none, 8B products.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for v in base st48 st96 base st48 st96; do
  if [ $v = base ]; then so=""; else so=ablib/_kernels_$v.so; fi
  echo "## $v" >> gpurun_out/r6s_bench.log
  FT_KERNELS_SO=$so timeout -k 10 300 python -u scripts/gemm_f32_bench.py 2>&1 | grep llama3 >> gpurun_out/r6s_bench.log || exit 1
done
cat gpurun_out/r6s_bench.log
