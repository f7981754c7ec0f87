#!/bin/bash
# Round-5 probe: five waves per SIMD (a 7-slot register file, 96 VGPRs, four
# LDS regions = 32 KiB per block) against C2's four-wave default (11 slots),
# alternated, two rounds; round 1 of the 7-slot build runs the oracle
# self-check.  The library (built in the container from a private copy of
# csrc/):
#   python -c "from mythril_amd import build as B; B.LAYOUTS[7] = (
#       'mythril_amd/lib/ab/libmythgpu_nreg7.so', ('MG_NREG_OVERRIDE=7',
#       'MG_ASM_WAVES_PER_SIMD=5', 'MG_LDS_SLOTS_DEFAULT=4')); B.build_layout(7, force=True)"
cd $GRAFT_REPO_ROOT || exit 1
D=gpurun_out/nreg7 && mkdir -p $D
( while true; do date >> $D/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
summ() { python -c "
import json,sys; t=open('$1').read(); d=json.loads(t[t.index('{'):])
print('%-22s value %.1f G  frac %.4f  kernel_ms %.2f  %s  bad %s' % ('$1'.split('/')[-1], d['value']/1e9, d['roofline']['frac'], d['roofline']['kernel_ms'], d['config']['register_layout'], (d.get('selfcheck') or {}).get('mismatches')))"; }
B="timeout -k 10 400 python -u bench.py --steps 3 --warmup 1"
NB="--no-cpu-baseline"
A7="env MYTHGPU_NREG=7 MYTHGPU_LIB=$PWD/mythril_amd/lib/ab/libmythgpu_nreg7.so MYTHGPU_LDS_SLOTS=4"
for R in 1 2; do
  $B $NB > $D/c2_r11_$R.log 2>&1 || { tail -20 $D/c2_r11_$R.log; exit 1; }
  summ $D/c2_r11_$R.log
  C=$NB; [ $R = 1 ] && C=
  $A7 $B $C > $D/c2_r7_$R.log 2>&1 || { tail -20 $D/c2_r7_$R.log; exit 1; }
  summ $D/c2_r7_$R.log
done
echo nreg7-ok
