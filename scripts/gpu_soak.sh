#!/bin/bash
# Soak runs (stability evidence): GPT-2-medium 3000 steps with an async checkpoint every 200 steps
# (BASELINE config 3 on one GPU) under the whole-step HIP graph; Llama-3-8B 600 steps.
export TMPDIR=/tmp
mkdir -p gpurun_out/soak
CK=/tmp/soakck; rm -rf $CK; mkdir -p $CK
W=$PWD/gpurun_out/soak; printf '#!/bin/bash\necho "Submitted batch job 1"\n' > $W/sbatch; chmod +x $W/sbatch
export PATH=$W:$PATH WORKDIR=$W
SLURM_JOB_ID=840001 timeout -k 10 500 python train.py --model gpt2-medium --synthetic-data --sequence-length 2048 --batch-size 1 \
  --learning-rate 5e-5 --lr-warmup-steps 100 --training-steps 3000 --save-every 200 --hip-graph --logging-frequency 100 \
  --checkpoint-path $CK > gpurun_out/soak/gpt2m_save_every_200.out 2>&1 || exit $?
rm -rf $CK; mkdir -p $CK
SLURM_JOB_ID=840002 timeout -k 10 500 python train.py --synthetic-data --sequence-length 2048 --batch-size 1 \
  --learning-rate 5e-5 --lr-warmup-steps 100 --training-steps 600 --logging-frequency 50 \
  --checkpoint-path $CK > gpurun_out/soak/llama8b_600.out 2>&1 || exit $?
rm -rf $CK
