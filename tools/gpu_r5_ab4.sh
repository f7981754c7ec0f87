#!/bin/bash
# Round-5 alternated A/B, fourth set (two rounds, the in-tree build first):
# C3 / C4 / C5, the calldata word's per-limb prefix mask against
# MYTHGPU_CDWX_PREFIX=0 (mythril_amd/lib/ab/libmythgpu_cdwxoff.so).
cd $GRAFT_REPO_ROOT || exit 1
D=gpurun_out/ab_r5d && mkdir -p $D
( while true; do date >> $D/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
summ() { python -c "
import json,sys; t=open('$1').read(); d=json.loads(t[t.index('{'):])
print('%-22s value %.1f G  frac %.4f  kernel_ms %.2f' % ('$1'.split('/')[-1], d['value']/1e9, d['roofline']['frac'], d['roofline']['kernel_ms']))"; }
B="timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
AB=mythril_amd/lib/ab
for R in 1 2; do
  for W in c3 c4 c5; do
    $B --workload $W > $D/${W}_new_$R.log 2>&1 || { tail -20 $D/${W}_new_$R.log; exit 1; }
    summ $D/${W}_new_$R.log
    MYTHGPU_CDWX_PREFIX=0 MYTHGPU_LIB=$AB/libmythgpu_cdwxoff.so $B --workload $W > $D/${W}_cdwxoff_$R.log 2>&1 || { tail -20 $D/${W}_cdwxoff_$R.log; exit 1; }
    summ $D/${W}_cdwxoff_$R.log
  done
done
echo ab-ok
