#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S pytest_gpu 500 python -m pytest tests -m gpu -x -q || exit 1
$S smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
$S b_def 300 python bench.py --steps 10 --warmup 3 || exit 1
CK=/tmp/ftck; rm -rf $CK; mkdir -p $CK
W=$PWD/gpurun_out/ftwd; mkdir -p $W
printf '#!/bin/bash\necho "$@" >> %s/sbatch_calls.txt\necho "Submitted batch job 777"\n' $W > $W/sbatch; chmod +x $W/sbatch
export PATH=$W:$PATH WORKDIR=$W
L8="--synthetic-data --sequence-length 2048 --batch-size 1 --checkpoint-path $CK --logging-frequency 5"
# sharded writer protocol on a 1-rank RCCL+gloo group, Llama-3-8B, ZeRO-1 forced
FT_FORCE_DIST=1 FT_SHARDED_CKPT=1 SLURM_JOB_ID=820001 $S llama_sharded 600 python train.py $L8 --dp-mode zero1 --training-steps 100 --raise-error --error-step 12 || exit 1
FT_FORCE_DIST=1 SLURM_JOB_ID=820002 $S llama_sharded_resume 600 python train.py $L8 --dp-mode zero1 --training-steps 16 --checkpoint-id 820001 || exit 1
python -c "import torch; c=torch.load('/tmp/ftck/checkpoint_820001.ckpt', map_location='cpu', weights_only=True, mmap=True); print('loaded', c['training_step'], len(c['model']), c['meta']['world_size'])" > gpurun_out/sharded_check.log 2>&1
cat gpurun_out/sharded_check.log
