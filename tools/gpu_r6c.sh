#!/bin/bash
# Round 6 (c): recall on the completed labels, then the schedule-choice A/B.
# A failing recall assertion (pytest exit 1) does not stop the A/B; anything
# else (a crash, a time limit) does.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6c
timeout -k 10 600 python -u -m pytest tests/test_gpu_recall.py -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/r6c/recall.log 2>&1
RC=$?
grep -E "recall c|passed|failed" gpurun_out/r6c/recall.log
if [ $RC -ne 0 ] && [ $RC -ne 1 ]; then tail -30 gpurun_out/r6c/recall.log; exit 1; fi
bash tools/gpu_r6_sched_ab.sh
