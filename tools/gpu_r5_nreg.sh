#!/bin/bash
# Round-5 probe: four waves per SIMD (an 11-slot register file, 128 VGPRs,
# five LDS regions = 40 KiB per block) against the default three waves
# (16 slots, 168 VGPRs, six regions), alternated, two rounds.  Each
# configuration assembles its images once, into its own cache directory
# (the image key does not carry the slot count).
# The 11-slot library (built in the container; the build regenerates the
# tracked mg_interp_gfx950.inc, so rebuild the default library after it):
#   MYTHGPU_NREG=11 python -c "from mythril_amd import build; build.build(force=True,
#       out='mythril_amd/lib/ab/libmythgpu_nreg11.so',
#       defines=['MG_NREG_OVERRIDE=11', 'MG_ASM_WAVES_PER_SIMD=4'])"
#   python -c "import __graft_entry__ as g; g.build()"
cd $GRAFT_REPO_ROOT || exit 1
D=gpurun_out/nreg_r5 && mkdir -p $D
( while true; do date >> $D/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
summ() { python -c "
import json,sys; t=open('$1').read(); d=json.loads(t[t.index('{'):])
print('%-22s value %.1f G  frac %.4f  kernel_ms %.2f  bad %s' % ('$1'.split('/')[-1], d['value']/1e9, d['roofline']['frac'], d['roofline']['kernel_ms'], (d.get('selfcheck') or {}).get('mismatches')))"; }
B="timeout -k 10 400 python -u bench.py --steps 3 --warmup 1"
NB="--no-cpu-baseline"
A11="env MYTHGPU_NREG=11 MYTHGPU_LIB=$PWD/mythril_amd/lib/ab/libmythgpu_nreg11.so MYTHGPU_LDS_SLOTS=5 MYTHGPU_JIT_CACHE=/tmp/jc_nreg11"
A16="env MYTHGPU_JIT_CACHE=/tmp/jc_nreg16"
for R in 1 2; do
  for W in c3 c5 c2; do
    $A16 $B $NB --workload $W > $D/${W}_r16_$R.log 2>&1 || { tail -20 $D/${W}_r16_$R.log; exit 1; }
    summ $D/${W}_r16_$R.log
    C=$NB; [ $R = 1 ] && C=  # round 1: oracle self-check of the 11-slot output
    $A11 $B $C --workload $W > $D/${W}_r11_$R.log 2>&1 || { tail -20 $D/${W}_r11_$R.log; exit 1; }
    summ $D/${W}_r11_$R.log
  done
done
echo nreg-ok
