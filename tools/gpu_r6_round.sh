#!/bin/bash
# Round 6 GPU check: the -m gpu suite, smoke(), the default bench line (C2,
# layout chosen per batch), the C3 / C5 lines, and the search bench (cold
# get_model latency with the host refutation).  Every step bounded, chained.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${TAG:-r6b}
( while true; do date >> gpurun_out/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 950 --timeout-method thread --durations=15 > gpurun_out/${T}_tests.log 2>&1 || { tail -60 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
for W in c2 c3 c5; do
  timeout -k 10 600 python -u bench.py --workload $W > gpurun_out/${T}_bench_$W.log 2>&1 || { tail -20 gpurun_out/${T}_bench_$W.log; exit 1; }
  python -c "
import json; t=open('gpurun_out/${T}_bench_$W.log').read(); d=json.loads(t[t.rindex('{\"metric\"'):])
print('$W', '%.1f G' % (d['value']/1e9), 'frac %.3f' % d['roofline']['frac'], d['config']['register_layout'], 'selfcheck', d.get('selfcheck', {}).get('mismatches'))"
done
timeout -k 10 600 python -u tools/search_bench.py --skip-corpus > gpurun_out/${T}_search.log 2>&1 || { tail -20 gpurun_out/${T}_search.log; exit 1; }
echo round-ok
