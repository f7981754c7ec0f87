#!/bin/bash
# Generic generator A/B on the compiled-program bench: the in-tree library
# against an alternative library built with a generator knob flipped
# (mythril_amd/lib/ab/*.so), alternated, two rounds.  asmgen reads the knob
# and also renders the compiled programs, so each run's image matches its
# library.
#   usage: [BENCH_ARGS="--workload c3"] bash tools/gpu_ab.sh <tag> <alt library> <KNOB=value> [...]
# e.g.   bash tools/gpu_ab.sh cmp mythril_amd/lib/ab/libmythgpu_cmpold.so MYTHGPU_CMP64=0
cd $GRAFT_REPO_ROOT || exit 1
TAG=$1; ALT=$2; shift 2
D=gpurun_out/ab_$TAG && mkdir -p $D
summ() { python -c "
import json,sys; t=open('$1').read(); d=json.loads(t[t.index('{'):])
print('%-16s value %.1f G  frac %.4f  kernel_ms %.2f' % ('$1'.split('/')[-1], d['value']/1e9, d['roofline']['frac'], d['roofline']['kernel_ms']))"; }
for R in 1 2; do
  L=$D/new_$R.log
  timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $L 2>&1 || { tail -20 $L; exit 1; }
  summ $L
  L=$D/old_$R.log
  env "$@" MYTHGPU_LIB=$ALT timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $L 2>&1 || { tail -20 $L; exit 1; }
  summ $L
done
echo ab-ok
