#!/bin/bash
#SBATCH --job-name=ftamd_train
#SBATCH --nodes=1
#SBATCH --ntasks-per-node=1
#SBATCH --gpus-per-node=1
#SBATCH --time=00:06:00
#SBATCH --output=logs/output_%j.out
#SBATCH --cpus-per-task=16
#SBATCH --signal=USR1@120
#SBATCH --no-requeue
# Same contract as the reference's train.sh (reference train.sh:1-30):
#   * Slurm sends SIGUSR1 120 s before the time limit; train.py saves a checkpoint
#     and resubmits this script with its own job id as $1;
#   * a resubmitted job passes $1 on as --checkpoint-id and resumes from it.
# For data parallelism set --ntasks-per-node / --gpus-per-node to N (one task per
# MI355X); train.py reads SLURM_PROCID / SLURM_LOCALID / SLURM_NTASKS.
# Site-specific lines (account, partition, container) go here.

TRAINING_CMD=" --sequence-length 2048 \
               --batch-size 1 \
               --learning-rate 5e-5 \
               --lr-warmup-steps 100 \
               --training-steps 1000 \
               --raise-error \
               --error-step 600 \
               ${EXTRA_TRAINING_ARGS}"

if [ -n "$1" ]; then
    TRAINING_CMD="$TRAINING_CMD \
     --checkpoint-id $1"
fi
export WORKDIR="${WORKDIR:-${SLURM_SUBMIT_DIR:-$PWD}}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
export MASTER_ADDR="${MASTER_ADDR:-127.0.0.1}"
export MASTER_PORT="${MASTER_PORT:-$((20000 + ${SLURM_JOB_ID:-0} % 20000))}"

exec srun --unbuffered python $WORKDIR/train.py $TRAINING_CMD
