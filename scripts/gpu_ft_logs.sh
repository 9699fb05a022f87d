#!/bin/bash
# MI355X fault-tolerance evidence (mirrors the reference's logs/: timeout -> resume -> error; cancel):
#  1) BASELINE config 2: GPT-2-small seq 2048, SIGUSR1 -> save -> sbatch resubmit chain x3 through train.sh
#     (Slurm emulator), whole-step HIP graph
#  2) BASELINE config 4 (data path): the IterableParquetDataset (byte tokenizer, generated parquet) on the
#     GPT-2-medium preset, SIGUSR1 mid-shard -> save -> resume chain x3 (the 8B state would need 2 x 48 GB of disk)
#  3) Llama-3-8B seq 2048: error-injection save (48 GB), resume from it, SIGTERM cancel
export TMPDIR=/tmp
mkdir -p gpurun_out/logs
S=scripts/gpu_check.sh
timeout -k 10 300 python -c "import torch; torch.zeros(1, device='cuda')" || exit 1   # page the image in
CK=/tmp/ftck; rm -rf $CK; mkdir -p $CK
$S chain_gpt2s 600 python benchmarks/preempt_chain.py --jobs 3 --time 60 --signal-lead 20 --checkpoint-path $CK --log-dir $PWD/gpurun_out/logs/chain_gpt2s -- --model gpt2-small --synthetic-data --hip-graph --logging-frequency 100 || exit 1
cp gpurun_out/chain_gpt2s.log gpurun_out/logs/ 2>/dev/null
rm -rf $CK; mkdir -p $CK
D=/tmp/ftdata; mkdir -p $D
python -c "import sys; sys.path.insert(0, 'tests'); from helpers import make_parquet; make_parquet('$D/train.parquet', n_docs=200000, seed=7)" || exit 1
$S chain_iter 600 python benchmarks/preempt_chain.py --jobs 3 --time 60 --signal-lead 20 --checkpoint-path $CK --log-dir $PWD/gpurun_out/logs/chain_iter -- --model gpt2-medium --dataset $D/train.parquet --iterable-dataset --tokenizer-name-or-path byte --vocab-size 131072 --logging-frequency 100 || exit 1
cp gpurun_out/chain_iter.log gpurun_out/logs/ 2>/dev/null
rm -rf $CK; mkdir -p $CK
W=$PWD/gpurun_out/ftwd; mkdir -p $W
printf '#!/bin/bash\necho "$@" >> %s/sbatch_calls.txt\necho "Submitted batch job 777"\n' $W > $W/sbatch; chmod +x $W/sbatch
export PATH=$W:$PATH WORKDIR=$W
L8="--synthetic-data --sequence-length 2048 --batch-size 1 --learning-rate 5e-5 --lr-warmup-steps 100 --checkpoint-path $CK --logging-frequency 5"
SLURM_JOB_ID=830001 $S llama_error 600 python train.py $L8 --training-steps 1000 --raise-error --error-step 40 || exit 1
cp gpurun_out/llama_error.log gpurun_out/logs/output_830001.out
SLURM_JOB_ID=830002 $S llama_resume 600 python train.py $L8 --training-steps 60 --checkpoint-id 830001 || exit 1
cp gpurun_out/llama_resume.log gpurun_out/logs/output_830002.out
rm -rf $CK; mkdir -p $CK
( SLURM_JOB_ID=830003 timeout -k 10 300 python train.py $L8 --training-steps 1000 > gpurun_out/logs/output_830003.out 2>&1 ) &
P=$!
for i in $(seq 1 240); do grep -q "Training step: 10 |" gpurun_out/logs/output_830003.out 2>/dev/null && break; sleep 1; done
kill -TERM $(pgrep -P $P python || echo $P) 2>/dev/null
wait $P; echo "cancel rc=$?"
tail -3 gpurun_out/logs/output_830003.out
rm -rf $CK $D
