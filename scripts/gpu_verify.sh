#!/bin/bash
# Round-end verification on one MI355X: GPU tests, smoke, headline bench, preset benches, and a
# rocprofv3 kernel-stats pass of the 8B step. Stops at the first failing step.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -20 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-400
for m in gpt2-small gpt2-medium; do
  timeout -k 10 200 python bench.py --model $m --graph --steps 50 --warmup 5 --no-ckpt > gpurun_out/bench_$m.log 2>&1 || exit 1
  tail -1 gpurun_out/bench_$m.log | cut -c1-300
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8b -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3 --no-ckpt > gpurun_out/prof8b.log 2>&1 || exit 1
tail -1 gpurun_out/prof8b.log | cut -c1-200
