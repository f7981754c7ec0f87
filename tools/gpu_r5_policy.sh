#!/bin/bash
# Leaf policy sweep on the round-5 kernel (spill placement in the translator
# makes spilled one-limb values cheap LDS dwords): C3 / C4 / C5 under the
# auto rule (their programs compile under "always") against "spill",
# "scratch"; C2 (auto: scratch2 for its heavy programs) against "spill".
cd $GRAFT_REPO_ROOT || exit 1
D=gpurun_out/pol_r5 && mkdir -p $D
( while true; do date >> $D/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
summ() { python -c "
import json,sys; t=open('$1').read(); d=json.loads(t[t.index('{'):])
print('%-22s value %.1f G  frac %.4f  kernel_ms %.2f' % ('$1'.split('/')[-1], d['value']/1e9, d['roofline']['frac'], d['roofline']['kernel_ms']))"; }
B="timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
for R in 1 2; do
for W in c3 c5 c4; do
  for P in auto spill scratch; do
    MYTHRIL_GPU_LEAF_REMAT=$P $B --workload $W > $D/${W}_${P}_$R.log 2>&1 || { tail -20 $D/${W}_${P}_$R.log; exit 1; }
    summ $D/${W}_${P}_$R.log
  done
done
for P in auto spill; do
  MYTHRIL_GPU_LEAF_REMAT=$P $B > $D/c2_${P}_$R.log 2>&1 || { tail -20 $D/c2_${P}_$R.log; exit 1; }
  summ $D/c2_${P}_$R.log
done
done
echo pol-ok
