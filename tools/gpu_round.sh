#!/bin/bash
# GPU round trip: full -m gpu parity suite, the search bench (per query
# shape), then the bench on C2 (no CPU leg) and on the C3 / C4 stand-in
# streams.  Each step has its own time limit and the script stops at the
# first failure.
# Usage: tools/gpu_round.sh <tag> [bench args...]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${1:-run}; shift
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; echo "gpu tests failed"; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -u tools/search_bench.py > gpurun_out/${TAG}_search.log 2>&1 || { tail -30 gpurun_out/${TAG}_search.log; echo "search bench failed"; exit 1; }
for W in c2 c3 c4; do
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --workload $W "$@" > gpurun_out/${TAG}_bench_$W.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_$W.log; echo "bench $W failed"; exit 1; }
  python -c "
import json,sys; t=open('gpurun_out/${TAG}_bench_$W.log').read(); d=json.loads(t[t.index('{'):])
print('$W value %.1f G  frac %.3f  kernel_ms %.1f' % (d['value']/1e9, d['roofline']['frac'], d['roofline']['kernel_ms']))"
done
