#!/bin/bash
# Leaf eviction policy A/B on the compiled-program bench (round 3: the
# compiled kernel is VALU-bound, so a leaf regenerated at its next use — ~45
# VALU of generator — may now cost more than an LDS / scratch spill and
# reload, which issue no VALU).  Policies alternated, two rounds.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/remat_jit
summ() { python -c "
import json,sys; t=open('$1').read(); d=json.loads(t[t.index('{'):])
print('%-24s value %.1f G  frac %.3f  kernel_ms %.1f' % ('$1'.split('/')[-1], d['value']/1e9, d['roofline']['frac'], d['roofline']['kernel_ms']))"; }
for R in 1 2; do
  for POL in "$@"; do
    L=gpurun_out/remat_jit/${POL}_$R.log
    MYTHRIL_GPU_LEAF_REMAT=$POL timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $L 2>&1 || { tail -20 $L; exit 1; }
    summ $L
  done
done
echo remat-ab-ok
