#!/bin/bash
# Round 6, session AA: no-GQA flash backward with the RoPE backward inside the dQ / dK-dV kernels (no
# rope_bwd_ pass): flash tests, model-level GPU tests, GPT-2 graph benches A/B (FT_FLASH_DIRECT_ROPE).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_flash_attn_gpu.py tests/test_w4_paths_gpu.py tests/test_kernels_gpu.py > gpurun_out/r6aa_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6aa_tests.log; [ $rc -eq 0 ] || exit $rc
for m in gpt2-small gpt2-medium; do
  for v in 1 0 1 0; do
    FT_FLASH_DIRECT_ROPE=$v timeout -k 10 300 python -u bench.py --model $m --vocab-size 50304 --graph --steps 50 --warmup 5 --no-ckpt > gpurun_out/r6aa_b.json 2>gpurun_out/r6aa_b.err || { tail -3 gpurun_out/r6aa_b.err; exit 1; }
    echo "$m direct_rope=$v $(python3 -c "import json;d=json.loads(open('gpurun_out/r6aa_b.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d.get('sclk_mhz_p50'))")" >> gpurun_out/r6aa_bench.log
  done
done
cat gpurun_out/r6aa_bench.log
