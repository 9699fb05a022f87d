#!/bin/bash
# Round-4 GPU session: kernel tests, GEMM bench, step A/B, headline bench, GPT-2 check.
# A failing test does not stop the measurements; a timeout / abort / segfault / GPU fault does.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
df -h /tmp . > gpurun_out/r4_df.txt
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[session] $name rc=$rc" | tee -a gpurun_out/r4_session.txt
  case $rc in 124|134|137|139) echo "[session] stopping after $name" | tee -a gpurun_out/r4_session.txt; exit $rc;; esac
  return 0
}
: > gpurun_out/r4_session.txt
step r4_tests 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gemm_w4t_gpu.py \
  tests/test_w4_paths_gpu.py tests/test_gemm_gpu.py tests/test_dtypes_gpu.py tests/test_flash_attn_gpu.py \
  -k "w4 or w4t or paths or flash"
step r4_gemm_bench 200 python -u scripts/gemm_w4t_bench.py
step r4_ab 600 python -u scripts/ab_step.py --knobs ${AB_KNOBS:-r4,dw} --rounds 2 --steps 8
step r4_bench 300 python -u bench.py --steps 20 --warmup 3 --no-ckpt
if [ -n "$PROF" ]; then  # per-kernel stats of the default 8B step (rocprofv3 kernel trace only)
  step r4_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4 -o run -- python3 bench.py --steps 5 --warmup 3 --no-ckpt
fi
if [ -n "$GPT2" ]; then
  step r4_gpt2_on 200 python -u bench.py --model gpt2-small --graph --steps 30 --warmup 5 --no-ckpt
  FT_W4_BWD=0 step r4_gpt2_off 200 python -u bench.py --model gpt2-small --graph --steps 30 --warmup 5 --no-ckpt
fi
exit 0
