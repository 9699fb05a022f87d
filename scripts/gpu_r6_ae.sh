#!/bin/bash
# Round 6, session AE: flash tests with the 3-kernel GQA form opt-in (default 4 kernels).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_flash_attn_gpu.py tests/test_w4_paths_gpu.py > gpurun_out/r6ae_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6ae_tests.log; exit $rc
