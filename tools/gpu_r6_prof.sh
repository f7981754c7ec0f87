#!/bin/bash
# Round 6 final evidence on one box: the recall test on the completed labels,
# rocprofv3 kernel-trace / HBM / SQ passes of the C2 / C3 / C4 / C5 bench
# configurations (tools/profile.sh, layout chosen per batch), then the four
# bench lines on the same box.  Each step bounded; the first failure ends it
# (a failing recall assertion, pytest exit 1, does not).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${TAG:-r6p}
( while true; do date >> gpurun_out/${T}_heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_recall.py -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_recall.log 2>&1
RC=$?
grep -E "recall c|passed|failed" gpurun_out/${T}_recall.log
if [ $RC -ne 0 ] && [ $RC -ne 1 ]; then tail -30 gpurun_out/${T}_recall.log; exit 1; fi
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
print('$W', '%.1f G' % (d['value']/1e9), 'frac %.3f' % r['frac'], 'traffic', r.get('traffic'), d['config']['register_layout'], 'selfcheck', d.get('selfcheck', {}).get('mismatches'))"
done
echo round-ok
