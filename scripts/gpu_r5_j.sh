#!/bin/bash
# Round 5, session J: w4 per-workgroup phase split (investigation build) + the production timeline.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
FT_KERNELS_SO=$GRAFT_REPO_ROOT/probe/_kernels_probe.so timeout -k 10 300 python -u scripts/w4_timeline.py --full > gpurun_out/r5j_w4_phases.log 2>&1; rc=$?
cat gpurun_out/r5j_w4_phases.log; exit $rc
