#!/bin/bash
# Bench A/B of a compiler knob (same library): the default bench line with
# and without an environment setting, alternated twice.
# usage: tools/gpu_ab_env.sh <tag> VAR=value
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=$1; KV=$2
for R in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_default_$R.log 2>&1 || exit 1
  env $KV timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_knob_$R.log 2>&1 || exit 1
done
for f in gpurun_out/${TAG}_*.log; do python -c "
import json; t=open('$f').read(); d=json.loads(t[t.index('{'):])
print('$f', 'value %.1f G  frac %.3f  kernel_ms %.1f' % (d['value']/1e9, d['roofline']['frac'], d['roofline']['kernel_ms']))"; done
