#!/bin/bash
# Round-5 A/B, sixth set: C2, bvumul_noovfl's all-overflow wave exit against
# MYTHGPU_UMULNO_FAST=0 (mythril_amd/lib/ab/libmythgpu_umulslow.so), two rounds.
cd $GRAFT_REPO_ROOT || exit 1
D=gpurun_out/ab_r5f && mkdir -p $D
( while true; do date >> $D/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
summ() { python -c "
import json,sys; t=open('$1').read(); d=json.loads(t[t.index('{'):])
print('%-22s value %.1f G  frac %.4f  kernel_ms %.2f' % ('$1'.split('/')[-1], d['value']/1e9, d['roofline']['frac'], d['roofline']['kernel_ms']))"; }
B="timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
for R in 1 2; do
  $B > $D/c2_new_$R.log 2>&1 || { tail -20 $D/c2_new_$R.log; exit 1; }
  summ $D/c2_new_$R.log
  MYTHGPU_UMULNO_FAST=0 MYTHGPU_LIB=mythril_amd/lib/ab/libmythgpu_umulslow.so $B > $D/c2_old_$R.log 2>&1 || { tail -20 $D/c2_old_$R.log; exit 1; }
  summ $D/c2_old_$R.log
done
echo ab-ok
