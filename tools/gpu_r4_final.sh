#!/bin/bash
# Round-4 final measurement set on one box: the -m gpu suite, the default
# bench line (CPU leg + self-check), C3 / C4 / C5 lines with their CPU legs,
# then rocprofv3 sets for every workload (tools/profile.sh).  Each GPU step
# has its own limit; the chain stops at the first failure.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
TAG=${1:-r4f}
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; echo "gpu tests failed"; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
fi
if [ -z "$SKIP_BENCH" ]; then
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench_c2.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_c2.log; exit 1; }
for W in c3 c4 c5; do
  timeout -k 10 600 python -u bench.py --workload $W > gpurun_out/${TAG}_bench_$W.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_$W.log; exit 1; }
done
fi
for W in $PROFILE_TAGS; do
  if [ "$W" = "c2" ]; then bash tools/profile.sh || { echo "profile c2 failed"; exit 1; }
  else PROF_TAG=$W bash tools/profile.sh --workload $W || { echo "profile $W failed"; exit 1; }
  fi
done
echo final-ok
