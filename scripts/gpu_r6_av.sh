#!/bin/bash
# Round 6, session AV: graph tests and a GPT-2-small graph bench after the queue guard.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_graphs_gpu.py tests/test_dp_rccl_gpu.py > gpurun_out/r6av_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r6av_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --model gpt2-small --vocab-size 50304 --graph --steps 50 --warmup 5 --no-ckpt 2>/dev/null | tail -1 | cut -c1-200
