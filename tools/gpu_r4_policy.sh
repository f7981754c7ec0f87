#!/bin/bash
# Leaf policy sweep on the final kernel (3-step bench lines, no CPU leg).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
D=gpurun_out/${1:-pol_r4} && mkdir -p $D
for W in c4 c3 c5 c2; do
for P in auto always scratch2 scratch; do
  L=$D/${W}_$P.log
  MYTHRIL_GPU_LEAF_REMAT=$P timeout -k 10 400 python -u bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline > $L 2>&1 || { tail -20 $L; exit 1; }
  python -c "
import json; t=open('$L').read(); d=json.loads(t[t.index('{'):].split(chr(10))[0])
print('%-4s %-9s value %.1f G  frac %.4f  kernel_ms %.2f' % ('$W', '$P', d['value']/1e9, d['roofline']['frac'], d['roofline']['kernel_ms']))"
done
done
echo policy-ok
