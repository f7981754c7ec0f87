#!/bin/bash
# Round-4 GPU check of the search path: the -m gpu suite, then the search
# bench (stand-in streams, get_model cold / stream phases).  Each GPU step
# has its own limit; the chain stops at the first failure.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
TAG=${1:-r4s}
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; echo "gpu tests failed"; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
fi
timeout -k 10 400 python -u tools/search_bench.py --skip-corpus > gpurun_out/${TAG}_search.log 2>&1 || { tail -20 gpurun_out/${TAG}_search.log; exit 1; }
echo search-ok
