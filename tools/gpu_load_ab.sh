#!/bin/bash
# get_model latency A/B of the host library (program upload path): the
# in-tree library against an alternative build (MYTHGPU_LIB), the search
# bench alternated, two rounds; prints the per-phase medians of each run.
#   usage: bash tools/gpu_load_ab.sh <tag> <alt library>
cd $GRAFT_REPO_ROOT || exit 1
TAG=$1; ALT=$2
D=gpurun_out/load_ab_$TAG && mkdir -p $D
summ() { python -c "
import json; t=open('$1').read(); d=json.loads(t[t.rindex('{\"device'):])
for w in ('c1','c3','c4'):
    for k in ('get_model','get_model_stream'):
        g=d['shapes'][w][k]; ph=g['phase_ms_per_query']
        print('%-10s %-3s %-16s median %6.2f ms  load %.3f  search %.3f  compile %.3f' % ('$1'.split('/')[-1][:-4], w, k, g['median_ms'], ph['load'], ph['search'], ph['compile']))"; }
for R in 1 2; do
  L=$D/new_$R.log
  timeout -k 10 400 python -u tools/search_bench.py > $L 2>&1 || { tail -20 $L; exit 1; }
  summ $L
  L=$D/old_$R.log
  MYTHGPU_LIB=$ALT timeout -k 10 400 python -u tools/search_bench.py > $L 2>&1 || { tail -20 $L; exit 1; }
  summ $L
done
echo load-ab-ok
