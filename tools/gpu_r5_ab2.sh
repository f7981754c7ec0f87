#!/bin/bash
# Round-5 alternated A/Bs, second set (two rounds, the in-tree build first;
# each alternative differs from it by ONE knob):
#   C2: two-limb short division (3-by-2 steps) against MYTHGPU_DIV_SHORT2=0
#       (mythril_amd/lib/ab/libmythgpu_short2off.so);
#   C2: the division's jump to digit 0 against MYTHGPU_DIV_J0=0
#       (mythril_amd/lib/ab/libmythgpu_divj0off.so);
#   C2 and C3: one-limb results read only at limb 0 left dirty (translator,
#       DC handler) against MYTHGPU_DIRTY_DC=0 (same library).
# asmgen reads the knobs and also renders the compiled programs, so each
# run's image matches its library.
cd $GRAFT_REPO_ROOT || exit 1
D=gpurun_out/ab_r5b && mkdir -p $D
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
  MYTHGPU_DIV_SHORT2=0 MYTHGPU_LIB=$AB/libmythgpu_short2off.so $B > $D/c2_s2off_$R.log 2>&1 || { tail -20 $D/c2_s2off_$R.log; exit 1; }
  summ $D/c2_s2off_$R.log
  MYTHGPU_DIV_J0=0 MYTHGPU_LIB=$AB/libmythgpu_divj0off.so $B > $D/c2_j0off_$R.log 2>&1 || { tail -20 $D/c2_j0off_$R.log; exit 1; }
  summ $D/c2_j0off_$R.log
  MYTHGPU_DIRTY_DC=0 $B > $D/c2_dirtyoff_$R.log 2>&1 || { tail -20 $D/c2_dirtyoff_$R.log; exit 1; }
  summ $D/c2_dirtyoff_$R.log
  $B --workload c3 > $D/c3_new_$R.log 2>&1 || { tail -20 $D/c3_new_$R.log; exit 1; }
  summ $D/c3_new_$R.log
  MYTHGPU_DIRTY_DC=0 $B --workload c3 > $D/c3_dirtyoff_$R.log 2>&1 || { tail -20 $D/c3_dirtyoff_$R.log; exit 1; }
  summ $D/c3_dirtyoff_$R.log
done
echo ab-ok
