#!/bin/bash
# Round-4 GPU check after a kernel change: the -m gpu suite (unless
# SKIP_TESTS), then one bench line per workload in $WORKLOADS (default
# "c2 c3 c4 c5"; --steps 3, no CPU leg).  Each GPU step has its own limit;
# the chain stops at the first failure.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
TAG=${1:-r4l}
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; echo "gpu tests failed"; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
fi
for W in ${WORKLOADS:-c2 c3 c4 c5}; do
  L=gpurun_out/${TAG}_bench_$W.log
  timeout -k 10 500 python -u bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline > $L 2>&1 || { tail -20 $L; exit 1; }
  python -c "
import json; t=open('$L').read(); d=json.loads(t[t.index('{\"metric'):])
print('$W value %.1f G frac %.4f kernel_ms %.2f' % (d['value']/1e9, d['roofline']['frac'], d['roofline']['kernel_ms']))"
done
echo lines-ok
