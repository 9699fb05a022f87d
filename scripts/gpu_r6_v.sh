#!/bin/bash
# Round 6, session V: full GPU suite + smoke + bench (no arguments) after the epilogue swizzle and the
# fp32 GEMM; the kernel stats of an fp32 GPT-2-small step (the fp32 GEMMs on gemm_f32).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6v_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6v_gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6v_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r6v_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r6v_bench_noargs.log 2>&1 || exit 1
tail -1 gpurun_out/r6v_bench_noargs.log | cut -c1-300
rm -rf gpurun_out/r6v_prof32
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6v_prof32 -o run --output-format csv -- python3 scripts/ab_step.py --model gpt2-small --vocab-size 50304 --dtype fp32 --knobs "" --rounds 1 --steps 5 --warmup 2 > gpurun_out/r6v_prof32.log 2>&1 || exit 1
python scripts/prof_summary.py $(find gpurun_out/r6v_prof32 -name "run_kernel_stats.csv" | head -1) "fp32 GPT-2-small step (vocab 50304), GEMMs on gemm_f32: scripts/ab_step.py --dtype fp32, 7 steps incl. warmup" 7 > gpurun_out/r6v_gpt2s_fp32_kernel_stats.md
head -20 gpurun_out/r6v_gpt2s_fp32_kernel_stats.md
rm -rf gpurun_out/r6v_prof32
