#!/bin/bash
# Round 5, session E: DP HIP-graph tests (1-rank RCCL), GPT-2-small / 8B kernel traces at HEAD.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/prof_g2s gpurun_out/prof_8b_e
timeout -k 10 600 python -u -m pytest tests/test_dp_rccl_gpu.py tests/test_graphs_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5e_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5e_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g2s -o run --output-format csv -- python3 bench.py --model gpt2-small --graph --vocab-size 50304 --steps 20 --warmup 3 --no-ckpt > gpurun_out/prof_g2s.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_8b_e -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3 --no-ckpt > gpurun_out/prof_8b_e.log 2>&1 || exit 1
echo done
