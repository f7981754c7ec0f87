#!/bin/bash
# A/B (round 6): the compiler's schedule choice (best of source order and the
# sink-driven order per program, the default) against source order only
# (MYTHRIL_GPU_SCHEDULE_CHOICE=0).  Both through the Python specification
# compiler (MYTHRIL_GPU_COMPILER=py: it emits the native compiler's programs)
# so the knob applies; default bench lines, alternated twice.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/sched2
D=gpurun_out/sched2
( while true; do date >> $D/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
export MYTHRIL_GPU_COMPILER=py
summ() { python -c "
import json; t=open('$1').read(); d=json.loads(t[t.rindex('{\"metric\"'):])
print('%-28s %.1f G  kernel %.2f ms  %s' % ('$1'.split('/')[-1], d['value']/1e9, d['roofline']['kernel_ms'], d['config']['register_layout']))"; }
for R in 1 2; do
 for W in c3 c4 c5 c2; do
  for S in 1 0; do
   MYTHRIL_GPU_SCHEDULE_CHOICE=$S timeout -k 10 500 python -u bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline > $D/${W}_choice${S}_$R.log 2>&1 || { tail -20 $D/${W}_choice${S}_$R.log; exit 1; }
   summ $D/${W}_choice${S}_$R.log
  done
 done
done
echo sched-ok
