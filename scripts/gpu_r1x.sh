#!/bin/bash
# restore path: GPU test + 8B error-save / resume timing
export TMPDIR=/tmp
mkdir -p gpurun_out/logs
S=scripts/gpu_check.sh
$S restore_test 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "h2d or pinned" || exit 1
CK=/tmp/ftck; rm -rf $CK; mkdir -p $CK
W=$PWD/gpurun_out/ftwd; mkdir -p $W
printf '#!/bin/bash\necho "$@" >> %s/sbatch_calls.txt\necho "Submitted batch job 777"\n' $W > $W/sbatch; chmod +x $W/sbatch
export PATH=$W:$PATH WORKDIR=$W
L8="--synthetic-data --sequence-length 2048 --batch-size 1 --learning-rate 5e-5 --lr-warmup-steps 100 --checkpoint-path $CK --logging-frequency 5"
SLURM_JOB_ID=810021 $S llama_error 600 python train.py $L8 --training-steps 1000 --raise-error --error-step 20 || exit 1
cp gpurun_out/llama_error.log gpurun_out/logs/output_810021.out
SLURM_JOB_ID=810022 $S llama_resume 600 python train.py $L8 --training-steps 30 --checkpoint-id 810021 || exit 1
cp gpurun_out/llama_resume.log gpurun_out/logs/output_810022.out
FT_RESTORE_PREAD=0 SLURM_JOB_ID=810023 $S llama_resume_mmap 600 python train.py $L8 --training-steps 30 --checkpoint-id 810021 || exit 1
cp gpurun_out/llama_resume_mmap.log gpurun_out/logs/output_810023.out
df -h /tmp > gpurun_out/df.txt; mount | grep -E " /tmp | / " >> gpurun_out/df.txt
rm -rf $CK
