#!/bin/bash
# The translator's round-5 choices re-checked on the four-wave layout (C2):
# spill placement (MYTHGPU_SPILL_PLACE=0: the round-4 slot rule) and dirty
# one-limb results (MYTHGPU_DIRTY_DC=0), against the default, alternated.
cd $GRAFT_REPO_ROOT || exit 1
D=gpurun_out/w4_knobs && mkdir -p $D
( while true; do date >> $D/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
summ() { python -c "
import json,sys; t=open('$1').read(); d=json.loads(t[t.index('{'):])
print('%-22s value %.1f G  frac %.4f  kernel_ms %.2f  %s' % ('$1'.split('/')[-1], d['value']/1e9, d['roofline']['frac'], d['roofline']['kernel_ms'], d['config']['register_layout']))"; }
B="timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
for R in 1 2; do
  $B > $D/c2_default_$R.log 2>&1 || { tail -20 $D/c2_default_$R.log; exit 1; }
  summ $D/c2_default_$R.log
  MYTHGPU_SPILL_PLACE=0 $B > $D/c2_placeoff_$R.log 2>&1 || { tail -20 $D/c2_placeoff_$R.log; exit 1; }
  summ $D/c2_placeoff_$R.log
  MYTHGPU_DIRTY_DC=0 $B > $D/c2_dirtyoff_$R.log 2>&1 || { tail -20 $D/c2_dirtyoff_$R.log; exit 1; }
  summ $D/c2_dirtyoff_$R.log
done
echo knobs-ok
