#!/bin/bash
# Division normalisation-order A/B on the compiled-program bench: the
# in-tree library (dividend bits before limbs) against
# mythril_amd/lib/ab/libmythgpu_divold.so (limbs, then 17 limbs of bits),
# alternated, two rounds.  The knob is read by asmgen, which also renders
# the compiled programs, so each run's image matches its library.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/div_ab
summ() { python -c "
import json,sys; t=open('$1').read(); d=json.loads(t[t.index('{'):])
print('%-16s value %.1f G  frac %.4f  kernel_ms %.2f' % ('$1'.split('/')[-1], d['value']/1e9, d['roofline']['frac'], d['roofline']['kernel_ms']))"; }
for R in 1 2; do
  L=gpurun_out/div_ab/new_$R.log
  timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $L 2>&1 || { tail -20 $L; exit 1; }
  summ $L
  L=gpurun_out/div_ab/old_$R.log
  MYTHGPU_DIV_BITS_FIRST=0 MYTHGPU_LIB=mythril_amd/lib/ab/libmythgpu_divold.so timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $L 2>&1 || { tail -20 $L; exit 1; }
  summ $L
done
echo div-ab-ok
