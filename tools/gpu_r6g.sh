#!/bin/bash
# Round 6 (g): recall after the construction's refusals, the schedule-gate
# A/B (SCHEDULE_MIN_SCRATCH = 10 against source order, through the Python
# specification compiler), then the profiles and bench lines of the final
# tree (tools/gpu_r6_prof.sh without its recall step).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gate
T=${TAG:-r6g}
( while true; do date >> gpurun_out/${T}_heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_recall.py -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_recall.log 2>&1
RC=$?
grep -E "recall c|passed|failed" gpurun_out/${T}_recall.log
if [ $RC -ne 0 ] && [ $RC -ne 1 ]; then tail -30 gpurun_out/${T}_recall.log; exit 1; fi
summ() { python -c "
import json; t=open('$1').read(); d=json.loads(t[t.rindex('{\"metric\"'):])
print('%-28s %.1f G  kernel %.2f ms  %s' % ('$1'.split('/')[-1], d['value']/1e9, d['roofline']['kernel_ms'], d['config']['register_layout']))"; }
for R in 1 2; do
 for W in c3 c4 c5; do
  MYTHRIL_GPU_COMPILER=py timeout -k 10 500 python -u bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/gate/${W}_gate_$R.log 2>&1 || { tail -20 gpurun_out/gate/${W}_gate_$R.log; exit 1; }
  summ gpurun_out/gate/${W}_gate_$R.log
  MYTHRIL_GPU_COMPILER=py MYTHRIL_GPU_SCHEDULE_CHOICE=0 timeout -k 10 500 python -u bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/gate/${W}_source_$R.log 2>&1 || { tail -20 gpurun_out/gate/${W}_source_$R.log; exit 1; }
  summ gpurun_out/gate/${W}_source_$R.log
 done
done
echo gate-ok
bash tools/profile.sh || { echo "profile c2 failed"; exit 1; }
for W in c3 c4 c5; do
  PROF_TAG=$W bash tools/profile.sh --workload $W || { echo "profile $W failed"; exit 1; }
done
echo profiles-ok
for W in c2 c3 c4 c5; do
  timeout -k 10 600 python -u bench.py --workload $W > gpurun_out/${T}_bench_$W.log 2>&1 || { tail -20 gpurun_out/${T}_bench_$W.log; exit 1; }
  python -c "
import json; t=open('gpurun_out/${T}_bench_$W.log').read(); d=json.loads(t[t.rindex('{\"metric\"'):])
r=d['roofline']
print('$W', '%.1f G' % (d['value']/1e9), 'frac %.3f' % r['frac'], d['config']['register_layout'], 'selfcheck', d.get('selfcheck', {}).get('mismatches'))"
done
echo round-ok
