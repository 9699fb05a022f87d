#!/bin/bash
# MI355X fault-tolerance evidence, mirroring the reference's logs/ (timeout -> resume -> error; cancel):
#  1) GPT-2-medium seq 2048: SIGUSR1 -> save -> sbatch resubmit chain x3 through train.sh (Slurm emulator)
#  2) Llama-3-8B seq 2048: error-injection save (48 GB), resume from it, SIGTERM cancel
export TMPDIR=/tmp
mkdir -p gpurun_out/logs
S=scripts/gpu_check.sh
CK=/tmp/ftck; rm -rf $CK; mkdir -p $CK
$S chain_gpt2m 900 python benchmarks/preempt_chain.py --jobs 3 --time 75 --signal-lead 25 --checkpoint-path $CK -- --model gpt2-medium --synthetic-data --sequence-length 2048 --batch-size 1 --learning-rate 5e-5 --lr-warmup-steps 100 --logging-frequency 50 || exit 1
cp /tmp/ftlogs_*/output_*.out gpurun_out/logs/ 2>/dev/null
rm -rf $CK; mkdir -p $CK
W=$PWD/gpurun_out/ftwd; mkdir -p $W
printf '#!/bin/bash\necho "$@" >> %s/sbatch_calls.txt\necho "Submitted batch job 777"\n' $W > $W/sbatch; chmod +x $W/sbatch
export PATH=$W:$PATH WORKDIR=$W
L8="--synthetic-data --sequence-length 2048 --batch-size 1 --learning-rate 5e-5 --lr-warmup-steps 100 --checkpoint-path $CK --logging-frequency 5"
SLURM_JOB_ID=810001 $S llama_error 600 python train.py $L8 --training-steps 1000 --raise-error --error-step 40 || exit 1
cp gpurun_out/llama_error.log gpurun_out/logs/output_810001.out
SLURM_JOB_ID=810002 $S llama_resume 600 python train.py $L8 --training-steps 60 --checkpoint-id 810001 || exit 1
cp gpurun_out/llama_resume.log gpurun_out/logs/output_810002.out
rm -rf $CK; mkdir -p $CK
( SLURM_JOB_ID=810003 timeout -k 10 300 python train.py $L8 --training-steps 1000 > gpurun_out/logs/output_810003.out 2>&1 ) &
P=$!
for i in $(seq 1 240); do grep -q "Training step: 10 |" gpurun_out/logs/output_810003.out 2>/dev/null && break; sleep 1; done
kill -TERM $(pgrep -P $P python || echo $P) 2>/dev/null
wait $P; echo "cancel rc=$?"
tail -3 gpurun_out/logs/output_810003.out
