#!/bin/bash
# GPU: storage facts, 8B checkpoint-save timing, train.py fault-tolerance flow on the GPU.
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
(df -h / /tmp "$GRAFT_REPO_ROOT" /dev/shm; free -g; nproc) > gpurun_out/box.txt 2>&1
CK=${CK_DIR:-/tmp/ftck}
mkdir -p $CK
$S bench_8b_ckpt 600 python bench.py --steps 5 --warmup 2 --ckpt-dir $CK || exit 1
rm -rf $CK/*
W=$PWD/gpurun_out/ftwd; mkdir -p $W
printf '#!/bin/bash\necho "$@" >> %s/sbatch_calls.txt\necho "Submitted batch job 777"\n' $W > $W/sbatch; chmod +x $W/sbatch
export PATH=$W:$PATH WORKDIR=$W
COMMON="--model gpt2-small --synthetic-data --sequence-length 2048 --batch-size 1 --learning-rate 5e-5 --lr-warmup-steps 100 --checkpoint-path $CK --logging-frequency 10 --training-steps 61"
SLURM_JOB_ID=501 $S ft_a 300 python train.py $COMMON --raise-error --error-step 30 || exit 1
SLURM_JOB_ID=502 $S ft_b 300 python train.py $COMMON --raise-error --error-step 60 --checkpoint-id 501 || exit 1
SLURM_JOB_ID=503 $S ft_c 300 python train.py $COMMON --raise-error --error-step 60 || exit 1
$S ft_cmp 120 python - <<'PY' || exit 1
import torch
a = torch.load("/tmp/ftck/checkpoint_502.ckpt", map_location="cpu", weights_only=True, mmap=True)
b = torch.load("/tmp/ftck/checkpoint_503.ckpt", map_location="cpu", weights_only=True, mmap=True)
bad = [k for k in a["model"] if not torch.equal(a["model"][k], b["model"][k])]
print("resumed-vs-uninterrupted identical params:", not bad, "mismatched:", bad[:4])
d = max((a["model"][k].float() - b["model"][k].float()).abs().max().item() for k in a["model"])
print("max abs diff", d)
PY
