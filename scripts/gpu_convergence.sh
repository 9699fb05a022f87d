#!/bin/bash
# Does the MI355X kernel set learn like the plain path? Byte-level text (a generated parquet), the same
# seed and data order, two runs per model: the default kernels (w4 forward GEMMs with the RoPE / SwiGLU
# epilogues, hardware rcp/sqrt in AdamW and SwiGLU) vs hipBLASLt for every GEMM, the separate RoPE and
# SwiGLU kernels and IEEE division/sqrt (FT_GEMM_BLAS=1 FT_EXACT_MATH=1).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/conv
D=/tmp/convdata; mkdir -p $D
python -c "import sys; sys.path.insert(0, 'tests'); from helpers import make_parquet; make_parquet('$D/train.parquet', n_docs=200000, seed=7)" || exit 1
DATA="--dataset $D/train.parquet --iterable-dataset --tokenizer-name-or-path byte --vocab-size 131072 --sequence-length 2048 --batch-size 1"
run() {  # run <name> <timeout> <env...> -- <args>
  local name=$1 to=$2; shift 2
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 $to python train.py $DATA "$@" > gpurun_out/conv/$name.out 2>&1 || { tail -5 gpurun_out/conv/$name.out; exit 1; }
  grep "Training step" gpurun_out/conv/$name.out | tail -1 | cut -c1-160
}
L8="--learning-rate 1e-4 --lr-warmup-steps 50 --training-steps 400 --logging-frequency 10 --checkpoint-path /tmp/convck --save-every 0"
G2="--model gpt2-medium --hip-graph --learning-rate 3e-4 --lr-warmup-steps 100 --training-steps 2000 --logging-frequency 25 --checkpoint-path /tmp/convck --save-every 0"
run llama8b_default 240 FT_NONE=1 -- $L8
run llama8b_plain 240 FT_GEMM_BLAS=1 FT_EXACT_MATH=1 -- $L8
run gpt2m_default 240 FT_NONE=1 -- $G2
run gpt2m_plain 240 FT_GEMM_BLAS=1 FT_EXACT_MATH=1 -- $G2
{
  echo "# Convergence on MI355X: default kernels vs the plain path (scripts/gpu_convergence.sh)"
  echo
  C=gpurun_out/conv
  python scripts/convergence_compare.py "Llama-3-8B, byte-level parquet text, lr 1e-4, 400 steps" default $C/llama8b_default.out plain $C/llama8b_plain.out
  python scripts/convergence_compare.py "GPT-2-medium (HIP graph), lr 3e-4, 2000 steps" default $C/gpt2m_default.out plain $C/gpt2m_plain.out
} > gpurun_out/conv/summary.md 2>&1
rm -rf /tmp/convck $D
tail -4 gpurun_out/conv/summary.md
