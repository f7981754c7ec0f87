#!/bin/bash
# GPU round for the compiled-program path: the -m gpu suite (every bench
# unit on the interpreter and compiled), then bench.py on C2 interpreted /
# compiled (alternated) and C3 / C4 compiled.  Stops at the first failure.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export MYTHGPU_JIT_CACHE=/tmp/mg_jitcache
TAG=${1:-jit}; shift
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; echo "gpu tests failed"; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
summ() { python -c "
import json,sys; t=open('$1').read(); d=json.loads(t[t.index('{'):])
print('%-28s value %.1f G  frac %.3f  kernel_ms %.1f  jit_s %s' % ('$1'.split('/')[-1], d['value']/1e9, d['roofline']['frac'], d['roofline']['kernel_ms'], d.get('jit_s')))"; }
for R in 1 2; do
  timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --interp > gpurun_out/${TAG}_c2_interp_$R.log 2>&1 || { tail -20 gpurun_out/${TAG}_c2_interp_$R.log; exit 1; }
  summ gpurun_out/${TAG}_c2_interp_$R.log
  timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_c2_jit_$R.log 2>&1 || { tail -20 gpurun_out/${TAG}_c2_jit_$R.log; exit 1; }
  summ gpurun_out/${TAG}_c2_jit_$R.log
done
for W in c3 c4; do
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --workload $W > gpurun_out/${TAG}_${W}_jit.log 2>&1 || { tail -20 gpurun_out/${TAG}_${W}_jit.log; exit 1; }
  summ gpurun_out/${TAG}_${W}_jit.log
done
