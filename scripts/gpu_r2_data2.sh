#!/bin/bash
# hipBLASLt vs rocBLAS per 8B product; GPT-2 presets at larger per-GPU batch (MFU vs GEMM size).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; rm -f gpurun_out/gpt2_batch.log
timeout -k 10 300 python3 scripts/blas_backend_bench.py > gpurun_out/blas_backend.log 2>&1 || exit $?
for m in gpt2-small gpt2-medium; do
  for b in 1 4 8; do
    g="--graph"
    out=$(timeout -k 10 240 python3 bench.py --model $m --batch-size $b --steps 20 --warmup 4 --no-ckpt $g 2>/dev/null) || exit $?
    echo "$m batch $b $g: $(echo "$out" | grep -o '"ms_per_step": [0-9.]*\|"mfu_vs_2.5PF_dense": [0-9.]*\|"tokens_per_s_per_gpu": [0-9.]*' | tr '\n' ' ')" | tee -a gpurun_out/gpt2_batch.log
  done
done
