#!/bin/bash
# flash timing; bit-exact resume on the GPU with --deterministic (gpt2-small, seq 2048)
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S flash_bench 300 python scripts/flash_bench.py || exit 1
CK=/tmp/ftck; mkdir -p $CK
W=$PWD/gpurun_out/ftwd; mkdir -p $W
printf '#!/bin/bash\necho "$@" >> %s/sbatch_calls.txt\necho "Submitted batch job 777"\n' $W > $W/sbatch; chmod +x $W/sbatch
export PATH=$W:$PATH WORKDIR=$W
COMMON="--model gpt2-small --synthetic-data --sequence-length 2048 --batch-size 1 --learning-rate 5e-4 --lr-warmup-steps 10 --checkpoint-path $CK --logging-frequency 10 --training-steps 61"
SLURM_JOB_ID=601 $S det_a 300 python train.py $COMMON --raise-error --error-step 60 || exit 1
SLURM_JOB_ID=602 $S det_a2 300 python train.py $COMMON --raise-error --error-step 60 || exit 1
SLURM_JOB_ID=603 $S det_b 300 python train.py $COMMON --raise-error --error-step 25 || exit 1
SLURM_JOB_ID=604 $S det_c 300 python train.py $COMMON --raise-error --error-step 60 --checkpoint-id 603 || exit 1
$S det_cmp 120 python - <<'PY' || exit 1
import torch
L = lambda j: torch.load(f"/tmp/ftck/checkpoint_{j}.ckpt", map_location="cpu", weights_only=True, mmap=True)
a, a2, c = L(601), L(602), L(604)
def cmp(x, y):
    bad = [k for k in x["model"] if not torch.equal(x["model"][k], y["model"][k])]
    bado = [i for i in x["optimizer"]["state"] if not torch.equal(x["optimizer"]["state"][i]["exp_avg_sq"], y["optimizer"]["state"][i]["exp_avg_sq"])]
    return len(bad), len(bado)
print("run-to-run (601 vs 602) mismatched params/moments:", cmp(a, a2))
print("uninterrupted vs resumed (601 vs 604) mismatched params/moments:", cmp(a, c))
PY
