#!/bin/bash
# Round-5 check: C2 on the final library against the same sources built with
# MYTHGPU_CDWX_PREFIX=0 (mythril_amd/lib/ab/libmythgpu_cdwxoff.so): C2's
# programs have no calldata word, so only the interpreter image's layout
# differs.
cd $GRAFT_REPO_ROOT || exit 1
D=gpurun_out/ab_r5e && mkdir -p $D
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
  MYTHGPU_CDWX_PREFIX=0 MYTHGPU_LIB=mythril_amd/lib/ab/libmythgpu_cdwxoff.so $B > $D/c2_old_$R.log 2>&1 || { tail -20 $D/c2_old_$R.log; exit 1; }
  summ $D/c2_old_$R.log
done
echo ab-ok
