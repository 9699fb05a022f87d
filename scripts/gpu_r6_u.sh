#!/bin/bash
# Round 6, session U: the optimizer side stream (norm + AdamW) confined to every 4th / 2nd CU by a CU
# mask, same-process 8B step A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/ab_step.py --knobs cumask --rounds 4 --steps 10 > gpurun_out/r6u_ab_cumask.log 2>&1 || { tail -5 gpurun_out/r6u_ab_cumask.log; exit 1; }
grep "best\|final" gpurun_out/r6u_ab_cumask.log
timeout -k 10 600 python -u scripts/ab_step.py --knobs cumask2 --rounds 4 --steps 10 > gpurun_out/r6u_ab_cumask2.log 2>&1 || { tail -5 gpurun_out/r6u_ab_cumask2.log; exit 1; }
grep "best\|final" gpurun_out/r6u_ab_cumask2.log
