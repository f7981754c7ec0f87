#!/bin/bash
# Quick check of a kernel change: the -m gpu suite, then 3-step bench lines
# (no CPU leg) for the four workloads, twice, alternated.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
TAG=${1:-r4q}
D=gpurun_out/$TAG && mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; echo "gpu tests failed"; exit 1; }
tail -1 $D/tests.log
for R in 1 2; do
for W in c2 c3 c4 c5; do
  L=$D/${W}_$R.log
  timeout -k 10 400 python -u bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline > $L 2>&1 || { tail -20 $L; exit 1; }
  python -c "
import json; t=open('$L').read(); d=json.loads(t[t.index('{'):].split(chr(10))[0])
print('%-10s value %.1f G  frac %.4f  kernel_ms %.2f' % ('$W/$R', d['value']/1e9, d['roofline']['frac'], d['roofline']['kernel_ms']))"
done
done
echo quick-ok
