#!/bin/bash
# Llama-3-8B throughput at seq 4096 / 16384, and 32768 with every block recomputed (README rows).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for S in 4096 16384; do
  timeout -k 10 240 python bench.py --seq-len $S --steps 8 --warmup 3 --no-ckpt > gpurun_out/bench_s$S.log 2>&1 || { tail -5 gpurun_out/bench_s$S.log; exit 1; }
  tail -1 gpurun_out/bench_s$S.log | cut -c1-330
done
timeout -k 10 300 python bench.py --seq-len 32768 --activation-checkpointing -1 --steps 5 --warmup 2 --no-ckpt > gpurun_out/bench_s32768.log 2>&1 || { tail -5 gpurun_out/bench_s32768.log; exit 1; }
tail -1 gpurun_out/bench_s32768.log | cut -c1-330
