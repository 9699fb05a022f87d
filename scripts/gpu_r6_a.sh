#!/bin/bash
# Round 6, session A: (1) which collective breaks ZeRO-1 under HIP-graph capture (one child per
# case, faulthandler on); (2) the ZeRO-1 --graph bench with faulthandler; (3) train.py vs bench.py
# on one box (8B, seq 2048, default flags, synthetic data).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/capture_collectives_probe.py > gpurun_out/r6a_capture_probe.log 2>&1
echo "probe rc $?"; grep -E "^=== " gpurun_out/r6a_capture_probe.log
export FT_GRAPH_ZERO1=1 FT_FORCE_DIST=1 HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -X faulthandler -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --model tiny --vocab-size 4096 --seq-len 256 \
  --steps 3 --warmup 1 --bucket-mb 0.5 --dp-mode zero1 --no-ckpt --graph > gpurun_out/r6a_zero1_graph.log 2>&1
echo "zero1 graph rc $?"
unset FT_GRAPH_ZERO1 FT_FORCE_DIST
# product loop vs bench, alternated on this box
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-ckpt > gpurun_out/r6a_bench_$r.log 2>&1 || exit 1
  tail -1 gpurun_out/r6a_bench_$r.log | cut -c1-200
  mkdir -p /tmp/ck6 && rm -rf /tmp/ck6/*
  SLURM_JOB_ID=6000$r timeout -k 10 400 python -u train.py --synthetic-data --sequence-length 2048 --batch-size 1 \
    --learning-rate 5e-5 --lr-warmup-steps 100 --training-steps 160 --logging-frequency 10 \
    --checkpoint-path /tmp/ck6 > gpurun_out/r6a_train_$r.log 2>&1 || exit 1
  grep -E "Training step: (100|150|160) " gpurun_out/r6a_train_$r.log
done
