#!/bin/bash
# (round 5: the same chain at the round-5 HEAD; --prune-on-resume: the box's 79 GB disk holds one
# 48 GB checkpoint, so the predecessor's goes once the next job resumed -- --prune-consumed, which
# waits for the next job's own save, needs room for two: its first attempt failed with ENOSPC,
# profiles/ft_logs_r5/enospc_attempt/)
# BASELINE config 4 at the 8B scale on one MI355X: Llama-3-8B (seq 2048, batch 1) reading the
# IterableParquetDataset (byte tokenizer, generated parquet), SIGUSR1 -> save (48 GB) -> resubmit ->
# resume chain x3 through train.sh under the Slurm emulator, with state digests at every save and
# resume. The consumed checkpoint is deleted once the next job has resumed from it (--prune-consumed:
# the box has 79 GB of disk, one 8B checkpoint is 48 GB). The job logs stream into gpurun_out/ft_r5.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ft_r5
S=scripts/gpu_check.sh
timeout -k 10 300 python -c "import torch; torch.zeros(1, device='cuda')" || exit 1   # page the image in
CK=/tmp/ftck; rm -rf $CK; mkdir -p $CK
D=/tmp/ftdata; mkdir -p $D
timeout -k 10 300 python -c "import sys; sys.path.insert(0, 'tests'); from helpers import make_parquet; make_parquet('$D/train.parquet', n_docs=200000, seed=7)" || exit 1
$S chain_iter_8b_r5 900 python benchmarks/preempt_chain.py --jobs 3 --time ${FT_TIME:-100} --signal-lead ${FT_LEAD:-30} \
  --checkpoint-path $CK --prune-on-resume --log-dir $PWD/gpurun_out/ft_r5 -- --dataset $D/train.parquet --iterable-dataset \
  --tokenizer-name-or-path byte --vocab-size 131072 --sequence-length 2048 --batch-size 1 \
  --learning-rate 5e-5 --lr-warmup-steps 100 --logging-frequency 50 --state-digest || exit 1
cp gpurun_out/chain_iter_8b_r5.log gpurun_out/ft_r5/ 2>/dev/null
rm -rf $CK $D
