#!/bin/bash
# bit-exact resume + run-to-run determinism on the GPU with the current step (dW side stream,
# deterministic flash bwd, pipelined optimizer): gpt2-small default, gpt2-medium with TN dW for all GEMMs
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
W=$PWD/gpurun_out/ftwd; mkdir -p $W
printf '#!/bin/bash\necho "$@" >> %s/sbatch_calls.txt\necho "Submitted batch job 777"\n' $W > $W/sbatch; chmod +x $W/sbatch
export PATH=$W:$PATH WORKDIR=$W
run_set() {  # run_set <tag> <model> [env...]
  local tag=$1 model=$2; shift 2
  local CK=/tmp/ftck_$tag; rm -rf $CK; mkdir -p $CK
  local C="--model $model --synthetic-data --sequence-length 2048 --batch-size 1 --learning-rate 5e-4 --lr-warmup-steps 10 --checkpoint-path $CK --logging-frequency 10 --training-steps 61"
  env "$@" SLURM_JOB_ID=601 $S ${tag}_a 300 python train.py $C --raise-error --error-step 60 || return 1
  env "$@" SLURM_JOB_ID=602 $S ${tag}_a2 300 python train.py $C --raise-error --error-step 60 || return 1
  env "$@" SLURM_JOB_ID=603 $S ${tag}_b 300 python train.py $C --raise-error --error-step 25 || return 1
  env "$@" SLURM_JOB_ID=604 $S ${tag}_c 300 python train.py $C --raise-error --error-step 60 --checkpoint-id 603 || return 1
  CK=$CK TAG=$tag $S ${tag}_cmp 120 python - <<'PY' || return 1
import os, torch
ck = os.environ["CK"]
L = lambda j: torch.load(f"{ck}/checkpoint_{j}.ckpt", map_location="cpu", weights_only=True, mmap=True)
a, a2, c = L(601), L(602), L(604)
def cmp(x, y):
    bad = [k for k in x["model"] if not torch.equal(x["model"][k], y["model"][k])]
    bado = [i for i in x["optimizer"]["state"] if not torch.equal(x["optimizer"]["state"][i]["exp_avg_sq"], y["optimizer"]["state"][i]["exp_avg_sq"])]
    return len(bad), len(bado)
print(os.environ["TAG"], "run-to-run (601 vs 602) mismatched params/moments:", cmp(a, a2))
print(os.environ["TAG"], "uninterrupted vs resumed (601 vs 604) mismatched params/moments:", cmp(a, c))
PY
  rm -rf $CK
}
run_set small gpt2-small FT_DW_STREAM=1 || exit 1
run_set mediumtn gpt2-medium FT_DW_STREAM=1 FT_DW_TRANSPOSE=all || exit 1
