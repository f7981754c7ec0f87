#!/bin/bash
# Round-5 probe: the LDS spill tier at 8 regions (16 halves = 64 KiB per
# block: 2 blocks, 2 waves per SIMD) against the default 6 (52 KiB, 3 blocks)
# on the spill-heavy C3 / C5, alternated, two rounds.
cd $GRAFT_REPO_ROOT || exit 1
D=gpurun_out/lds8_r5 && mkdir -p $D
( while true; do date >> $D/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
summ() { python -c "
import json,sys; t=open('$1').read(); d=json.loads(t[t.index('{'):])
print('%-22s value %.1f G  frac %.4f  kernel_ms %.2f' % ('$1'.split('/')[-1], d['value']/1e9, d['roofline']['frac'], d['roofline']['kernel_ms']))"; }
B="timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
for R in 1 2; do
  for W in c3 c5; do
    $B --workload $W > $D/${W}_lds6_$R.log 2>&1 || { tail -20 $D/${W}_lds6_$R.log; exit 1; }
    summ $D/${W}_lds6_$R.log
    MYTHGPU_LDS_SLOTS=8 $B --workload $W > $D/${W}_lds8_$R.log 2>&1 || { tail -20 $D/${W}_lds8_$R.log; exit 1; }
    summ $D/${W}_lds8_$R.log
  done
done
echo lds-ok
