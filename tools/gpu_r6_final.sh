#!/bin/bash
# Round 6 close: the -m gpu suite, smoke(), the default bench line on the
# final tree, then the schedule-choice A/B (tools/gpu_r6_sched_ab.sh).
# Every step bounded; the first failure ends it.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${TAG:-r6f}
( while true; do date >> gpurun_out/${T}_heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 950 --timeout-method thread --durations=15 > gpurun_out/${T}_tests.log 2>&1 || { tail -60 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 || { tail -20 gpurun_out/${T}_bench.log; exit 1; }
tail -c 600 gpurun_out/${T}_bench.log
bash tools/gpu_r6_sched_ab.sh
