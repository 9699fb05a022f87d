#!/bin/bash
# background pinned preallocation: ckpt GPU tests, 8B error-save (48 GB) + resume through train.py
export TMPDIR=/tmp
mkdir -p gpurun_out/logs4
S=scripts/gpu_check.sh
$S pa_test 300 python -u -m pytest tests/test_ckpt_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
CK=/tmp/ftck; rm -rf $CK; mkdir -p $CK
W=$PWD/gpurun_out/ftwd4; mkdir -p $W
printf '#!/bin/bash\necho "$@" >> %s/sbatch_calls.txt\necho "Submitted batch job 777"\n' $W > $W/sbatch; chmod +x $W/sbatch
export PATH=$W:$PATH WORKDIR=$W
L8="--synthetic-data --sequence-length 2048 --batch-size 1 --learning-rate 5e-5 --lr-warmup-steps 100 --checkpoint-path $CK --logging-frequency 5"
SLURM_JOB_ID=820001 $S pa_error 600 python train.py $L8 --training-steps 1000 --raise-error --error-step 60 || exit 1
cp gpurun_out/pa_error.log gpurun_out/logs4/output_820001.out
SLURM_JOB_ID=820002 $S pa_resume 600 python train.py $L8 --training-steps 70 --checkpoint-id 820001 || exit 1
cp gpurun_out/pa_resume.log gpurun_out/logs4/output_820002.out
grep -h "Checkpoint /\|Resuming\|Training step: 6[05]" gpurun_out/logs4/*.out
