#!/bin/bash
# Round-4 GPU round trip: the -m gpu suite, the default bench line (CPU leg +
# self-check), the C5 all-contracts line, then rocprofv3 sets for the
# workloads in $PROFILE_TAGS ("c2" = the default bench, else --workload <w>).
# Each GPU step has its own time limit; the chain stops at the first failure.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
# long fixtures (oracle runs over every bench unit, image assembly) print
# nothing for minutes: keep a heartbeat file moving for gpurun's watchdog
( while true; do date >> gpurun_out/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
TAG=${1:-r4}
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; echo "gpu tests failed"; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
fi
if [ -z "$SKIP_BENCH" ]; then
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -c 600 gpurun_out/${TAG}_bench.log
timeout -k 10 600 python -u bench.py --workload c5 > gpurun_out/${TAG}_bench_c5.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_c5.log; exit 1; }
tail -c 600 gpurun_out/${TAG}_bench_c5.log
fi
for W in $PROFILE_TAGS; do
  if [ "$W" = "c2" ]; then bash tools/profile.sh || { echo "profile c2 failed"; exit 1; }
  else PROF_TAG=$W bash tools/profile.sh --workload $W || { echo "profile $W failed"; exit 1; }
  fi
done
echo r4-ok
