#!/bin/bash
# Round-5 alternated A/Bs, third set (two rounds, the in-tree build first;
# each alternative differs from it by ONE knob), C2:
#   a wave whose every divisor is zero skips the division, against
#       MYTHGPU_DIV_ZERO_EXIT=0 (mythril_amd/lib/ab/libmythgpu_zexitoff.so);
#   the reciprocal after the digit-0 test of a full-width-divisor wave,
#       against MYTHGPU_DIV_J0_LATE=0 (mythril_amd/lib/ab/libmythgpu_j0lateoff.so).
cd $GRAFT_REPO_ROOT || exit 1
D=gpurun_out/ab_r5c && mkdir -p $D
( while true; do date >> $D/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
summ() { python -c "
import json,sys; t=open('$1').read(); d=json.loads(t[t.index('{'):])
print('%-22s value %.1f G  frac %.4f  kernel_ms %.2f' % ('$1'.split('/')[-1], d['value']/1e9, d['roofline']['frac'], d['roofline']['kernel_ms']))"; }
B="timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
AB=mythril_amd/lib/ab
for R in 1 2; do
  $B > $D/c2_new_$R.log 2>&1 || { tail -20 $D/c2_new_$R.log; exit 1; }
  summ $D/c2_new_$R.log
  MYTHGPU_DIV_ZERO_EXIT=0 MYTHGPU_LIB=$AB/libmythgpu_zexitoff.so $B > $D/c2_zexitoff_$R.log 2>&1 || { tail -20 $D/c2_zexitoff_$R.log; exit 1; }
  summ $D/c2_zexitoff_$R.log
  MYTHGPU_DIV_J0_LATE=0 MYTHGPU_LIB=$AB/libmythgpu_j0lateoff.so $B > $D/c2_j0lateoff_$R.log 2>&1 || { tail -20 $D/c2_j0lateoff_$R.log; exit 1; }
  summ $D/c2_j0lateoff_$R.log
done
echo ab-ok
