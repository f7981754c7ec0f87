#!/bin/bash
# One box, one measurement set, chained so the first failure ends it:
#   tools/gpu_measure.sh <tag> <steps> [workloads]
# <steps>: comma list of tests,bench,profile,search
#   tests   - the -m gpu suite
#   bench   - the default bench line per workload (CPU leg + self-check)
#   profile - tools/profile.sh per workload (kernel trace, FETCH, WRITE, SQ)
#   search  - tools/search_bench.py
# workloads default to "c2 c3 c4 c5".  (Settings go on the command line:
# the box does not inherit this container's environment.)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
TAG=$1; STEPS=",$2,"; WL=${3:-c2 c3 c4 c5}
if [[ $STEPS == *,tests,* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; echo "gpu tests failed"; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
fi
if [[ $STEPS == *,bench,* ]]; then
  for W in $WL; do
    timeout -k 10 600 python -u bench.py --workload $W > gpurun_out/${TAG}_bench_$W.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_$W.log; echo "bench $W failed"; exit 1; }
  done
fi
if [[ $STEPS == *,profile,* ]]; then
  for W in $WL; do
    if [ "$W" = "c2" ]; then bash tools/profile.sh || { echo "profile c2 failed"; exit 1; }
    else PROF_TAG=$W bash tools/profile.sh --workload $W || { echo "profile $W failed"; exit 1; }
    fi
  done
fi
if [[ $STEPS == *,search,* ]]; then
  timeout -k 10 400 python -u tools/search_bench.py > gpurun_out/${TAG}_search.log 2>&1 || { tail -30 gpurun_out/${TAG}_search.log; echo "search bench failed"; exit 1; }
fi
echo measure-ok
