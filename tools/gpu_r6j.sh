#!/bin/bash
# Round 6 (j), the close: the -m gpu suite and smoke() on the final tree,
# then the profile passes and the four bench lines (tools/profile.sh,
# keyed traffic for profiles/traffic.json).  Every step bounded; the first
# failure ends it.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${TAG:-r6j}
( while true; do date >> gpurun_out/${T}_heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 850 --timeout-method thread --durations=10 > gpurun_out/${T}_tests.log 2>&1 || { tail -60 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
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
