#!/bin/bash
# Round 6, session K (evidence at HEAD): full GPU suite + smoke, bench.py as the driver runs it (no
# arguments), rocprofv3 kernel stats of the 8B step and of the GPT-2-medium graph step.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6k_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6k_gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6k_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r6k_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r6k_bench_noargs.log 2>&1 || exit 1
tail -1 gpurun_out/r6k_bench_noargs.log | cut -c1-300
rm -rf gpurun_out/r6k_prof8b gpurun_out/r6k_profgm
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r6k_prof8b -o run --output-format csv -- python3 bench.py --steps 8 --warmup 2 --no-ckpt > gpurun_out/r6k_prof8b.log 2>&1 || exit 1
python scripts/prof_summary.py $(find gpurun_out/r6k_prof8b -name "run_kernel_stats.csv" | head -1) "Llama-3-8B bench step at the end of round 6 (10 steps incl. 2 warmup)" 10 > gpurun_out/r6k_llama8b_kernel_stats.md
head -25 gpurun_out/r6k_llama8b_kernel_stats.md
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6k_profgm -o run --output-format csv -- python3 bench.py --model gpt2-medium --vocab-size 50304 --graph --steps 20 --warmup 3 --no-ckpt > gpurun_out/r6k_profgm.log 2>&1 || exit 1
python scripts/prof_summary.py $(find gpurun_out/r6k_profgm -name "run_kernel_stats.csv" | head -1) "GPT-2-medium vocab 50304 --graph, end of round 6 (23 steps incl. warmup)" 23 > gpurun_out/r6k_gpt2m_kernel_stats.md
head -12 gpurun_out/r6k_gpt2m_kernel_stats.md
rm -rf gpurun_out/r6k_prof8b gpurun_out/r6k_profgm
