#!/bin/bash
# The four-wave layout on C4 (the stream with the least spill traffic):
# MYTHGPU_NREG=11 against the 16-slot default, alternated, two rounds.
cd $GRAFT_REPO_ROOT || exit 1
D=gpurun_out/nreg_c4 && mkdir -p $D
( while true; do date >> $D/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
summ() { python -c "
import json,sys; t=open('$1').read(); d=json.loads(t[t.index('{'):])
print('%-22s value %.1f G  frac %.4f  kernel_ms %.2f  %s' % ('$1'.split('/')[-1], d['value']/1e9, d['roofline']['frac'], d['roofline']['kernel_ms'], d['config']['register_layout']))"; }
B="timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --workload c4"
for R in 1 2; do
  $B > $D/c4_r16_$R.log 2>&1 || { tail -20 $D/c4_r16_$R.log; exit 1; }
  summ $D/c4_r16_$R.log
  MYTHGPU_NREG=11 $B > $D/c4_r11_$R.log 2>&1 || { tail -20 $D/c4_r11_$R.log; exit 1; }
  summ $D/c4_r11_$R.log
done
echo nreg-c4-ok
