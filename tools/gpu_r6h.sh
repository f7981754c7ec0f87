#!/bin/bash
# Round 6 (h): the -m gpu suite, smoke(), the default bench line and the
# search bench on the final tree.  Every step bounded; the first failure
# ends it.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${TAG:-r6h}
( while true; do date >> gpurun_out/${T}_heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 950 --timeout-method thread --durations=15 > gpurun_out/${T}_tests.log 2>&1 || { tail -60 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 || { tail -20 gpurun_out/${T}_bench.log; exit 1; }
python -c "
import json; t=open('gpurun_out/${T}_bench.log').read(); d=json.loads(t[t.rindex('{\"metric\"'):])
r=d['roofline']
print('c2', '%.1f G' % (d['value']/1e9), 'frac %.3f' % r['frac'], 'traffic', r.get('traffic'), 'valu_active', r.get('valu_active'), 'selfcheck', d.get('selfcheck', {}).get('mismatches'))"
timeout -k 10 600 python -u tools/search_bench.py --skip-corpus > gpurun_out/${T}_search.log 2>&1 || { tail -20 gpurun_out/${T}_search.log; exit 1; }
echo round-ok
