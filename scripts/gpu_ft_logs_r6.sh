#!/bin/bash
# Round 6: BASELINE config 4 at the 8B scale, in the SAFE order on a box whose 79 GB disk holds one
# 48 GB checkpoint: two checkpoint tiers -- /tmp (the disk) and /dev/shm (host memory, 1.5 TB) --
# rotated per job (train.py --checkpoint-alt-path --prune-consumed): each job resumes from one tier,
# writes its own checkpoint to the other and deletes its predecessor's file only after its own is
# durable. benchmarks/preempt_chain.py samples both directories every 50 ms and reports the minimum
# number of complete checkpoints after the first save (must be >= 1). Llama-3-8B, seq 2048, batch 1,
# IterableParquetDataset (byte tokenizer, generated parquet), SIGUSR1 -> save -> resubmit -> resume x3,
# state digests at every save and resume. Job logs stream into gpurun_out/ft_r6.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ft_r6
S=scripts/gpu_check.sh
timeout -k 10 300 python -c "import torch; torch.zeros(1, device='cuda')" || exit 1   # page the image in
CK=/tmp/ftck; ALT=/dev/shm/ftck_r6; rm -rf $CK $ALT; mkdir -p $CK $ALT
D=/tmp/ftdata; mkdir -p $D
timeout -k 10 300 python -c "import sys; sys.path.insert(0, 'tests'); from helpers import make_parquet; make_parquet('$D/train.parquet', n_docs=200000, seed=7)" || exit 1
$S chain_iter_8b_r6 900 python benchmarks/preempt_chain.py --jobs 3 --time ${FT_TIME:-100} --signal-lead ${FT_LEAD:-30} \
  --checkpoint-path $CK --rotate $ALT --log-dir $PWD/gpurun_out/ft_r6 -- --dataset $D/train.parquet --iterable-dataset \
  --tokenizer-name-or-path byte --vocab-size 131072 --sequence-length 2048 --batch-size 1 \
  --learning-rate 5e-5 --lr-warmup-steps 100 --logging-frequency 50 --state-digest || exit 1
cp gpurun_out/chain_iter_8b_r6.log gpurun_out/ft_r6/ 2>/dev/null
ls -la $CK $ALT | tee gpurun_out/ft_r6/final_dirs.txt
rm -rf $CK $ALT $D
