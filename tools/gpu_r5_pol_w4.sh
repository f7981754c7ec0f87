#!/bin/bash
# Leaf policy sweep for C2 on the four-wave layout (bench's default for C2:
# 11 slots, five LDS regions): the auto rule against scratch2 / scratch /
# always, alternated, two rounds.
cd $GRAFT_REPO_ROOT || exit 1
D=gpurun_out/pol_w4 && mkdir -p $D
( while true; do date >> $D/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
summ() { python -c "
import json,sys; t=open('$1').read(); d=json.loads(t[t.index('{'):])
print('%-22s value %.1f G  frac %.4f  kernel_ms %.2f  %s' % ('$1'.split('/')[-1], d['value']/1e9, d['roofline']['frac'], d['roofline']['kernel_ms'], d['config']['register_layout']))"; }
B="timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
for R in 1 2; do
  for P in auto scratch2 scratch always; do
    MYTHRIL_GPU_LEAF_REMAT=$P $B > $D/c2_${P}_$R.log 2>&1 || { tail -20 $D/c2_${P}_$R.log; exit 1; }
    summ $D/c2_${P}_$R.log
  done
done
echo pol-ok
