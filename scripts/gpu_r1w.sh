#!/bin/bash
# full GPU suite, 8B error-save + resume timing (pinned-ring restore), bench, clean profile
export TMPDIR=/tmp
mkdir -p gpurun_out/logs
S=scripts/gpu_check.sh
$S gpu_tests 900 python -m pytest tests -m gpu -x -q || exit 1
CK=/tmp/ftck; rm -rf $CK; mkdir -p $CK
W=$PWD/gpurun_out/ftwd; mkdir -p $W
printf '#!/bin/bash\necho "$@" >> %s/sbatch_calls.txt\necho "Submitted batch job 777"\n' $W > $W/sbatch; chmod +x $W/sbatch
export PATH=$W:$PATH WORKDIR=$W
L8="--synthetic-data --sequence-length 2048 --batch-size 1 --learning-rate 5e-5 --lr-warmup-steps 100 --checkpoint-path $CK --logging-frequency 5"
SLURM_JOB_ID=810011 $S llama_error 600 python train.py $L8 --training-steps 1000 --raise-error --error-step 30 || exit 1
cp gpurun_out/llama_error.log gpurun_out/logs/output_810011.out
SLURM_JOB_ID=810012 $S llama_resume 600 python train.py $L8 --training-steps 45 --checkpoint-id 810011 || exit 1
cp gpurun_out/llama_resume.log gpurun_out/logs/output_810012.out
rm -rf $CK
$S bench 300 python bench.py --steps 20 --warmup 3 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$S prof_w 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_w -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --whole-buffer-optimizer || exit 1
