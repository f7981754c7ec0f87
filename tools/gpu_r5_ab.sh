#!/bin/bash
# Round-5 alternated A/Bs on one box (two rounds each, new build first):
#   spill placement (translator, mg_host.cpp place_spills) on C3 and C5
#     against MYTHGPU_SPILL_PLACE=0 (the round-4 slot rule);
#   the one-limb short division's branch over its second correction on C2
#     against the round-4 step (library built with MYTHGPU_DIV_SHORT_BRANCH=0
#     into mythril_amd/lib/ab/libmythgpu_divr4.so).
cd $GRAFT_REPO_ROOT || exit 1
D=gpurun_out/ab_r5 && mkdir -p $D
( while true; do date >> $D/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
summ() { python -c "
import json,sys; t=open('$1').read(); d=json.loads(t[t.index('{'):])
print('%-22s value %.1f G  frac %.4f  kernel_ms %.2f' % ('$1'.split('/')[-1], d['value']/1e9, d['roofline']['frac'], d['roofline']['kernel_ms']))"; }
B="timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
for R in 1 2; do
  for W in c3 c5; do
    $B --workload $W > $D/${W}_new_$R.log 2>&1 || { tail -20 $D/${W}_new_$R.log; exit 1; }
    summ $D/${W}_new_$R.log
    MYTHGPU_SPILL_PLACE=0 $B --workload $W > $D/${W}_old_$R.log 2>&1 || { tail -20 $D/${W}_old_$R.log; exit 1; }
    summ $D/${W}_old_$R.log
  done
  $B > $D/c2_new_$R.log 2>&1 || { tail -20 $D/c2_new_$R.log; exit 1; }
  summ $D/c2_new_$R.log
  MYTHGPU_DIV_SHORT_BRANCH=0 MYTHGPU_LIB=mythril_amd/lib/ab/libmythgpu_divr4.so $B > $D/c2_old_$R.log 2>&1 || { tail -20 $D/c2_old_$R.log; exit 1; }
  summ $D/c2_old_$R.log
done
echo ab-ok
