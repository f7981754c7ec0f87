#!/bin/bash
# Round 6: the -m gpu suite (now with the four-wave layout's whole-configuration
# parity, tests/test_gpu_layout.py), then smoke().
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${TAG:-r6a}
( while true; do date >> gpurun_out/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 950 --timeout-method thread --durations=15 > gpurun_out/${T}_tests.log 2>&1 || { tail -60 gpurun_out/${T}_tests.log; exit 1; }
tail -20 gpurun_out/${T}_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
echo tests-ok
