#!/bin/bash
# Instruction-cache counters of the interpreter (one PMC pass, 512 DAGs).
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_IFETCH SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVE_CYCLES SQ_INSTS_VALU --output-format csv -d gpurun_out/prof/ic -o ic -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --dags 512 > gpurun_out/prof/ic.log 2>&1 || { tail -5 gpurun_out/prof/ic.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof/ic/**/*counter_collection.csv", recursive=True)[0]
c = {}
for r in csv.DictReader(open(f)):
    if "mg_interp_asm<0>" in r["Kernel_Name"]:
        c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for k in sorted(c): print(k, "%.4g" % c[k])
PY
