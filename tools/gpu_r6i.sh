#!/bin/bash
# Round 6 (i): the compiled MUL's one-limb rows (asmgen.MUL_SHORT) — the
# whole-configuration parity of the C2 bench with them on, then an
# alternated A/B of the default C2 bench line (knob on / off, two rounds).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/mul
D=gpurun_out/mul
( while true; do date >> $D/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
MYTHGPU_MUL_SHORT=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_parity.py -x -v -s -k c2 --timeout 850 --timeout-method thread > $D/parity_on.log 2>&1 || { tail -40 $D/parity_on.log; exit 1; }
grep -E "passed|failed" $D/parity_on.log | tail -2
summ() { python -c "
import json; t=open('$1').read(); d=json.loads(t[t.rindex('{\"metric\"'):])
print('%-22s %.1f G  kernel %.2f ms  selfcheck %s' % ('$1'.split('/')[-1], d['value']/1e9, d['roofline']['kernel_ms'], d.get('selfcheck', {}).get('mismatches')))"; }
for R in 1 2; do
  for K in 1 0; do
    MYTHGPU_MUL_SHORT=$K timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D/c2_mul${K}_$R.log 2>&1 || { tail -20 $D/c2_mul${K}_$R.log; exit 1; }
    summ $D/c2_mul${K}_$R.log
  done
done
echo mul-ok
