#!/bin/bash
# Where the interpreter's wave time goes: two SQ counter passes (<= 8 SQ
# counters each) over the 512-DAG bench slice, summed per counter for the
# evaluation kernel.
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --dags 512 $@"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH --output-format csv -d gpurun_out/prof/st1 -o st1 -- python3 bench.py $ARGS > gpurun_out/prof/st1.log 2>&1 || { tail -5 gpurun_out/prof/st1.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC --output-format csv -d gpurun_out/prof/st2 -o st2 -- python3 bench.py $ARGS > gpurun_out/prof/st2.log 2>&1 || { tail -5 gpurun_out/prof/st2.log; exit 1; }
python3 - <<'PY'
import csv, glob, json
c = {}
for f in glob.glob("gpurun_out/prof/st*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mg_interp_asm<0>" in r["Kernel_Name"]:
            c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
w = c.get("SQ_WAVES", 1.0)
out = {k: v for k, v in sorted(c.items())}
out["per_wave"] = {k: v / w for k, v in sorted(c.items()) if k != "SQ_WAVES"}
print(json.dumps(out, indent=1))
json.dump(out, open("gpurun_out/prof/stalls.json", "w"), indent=1)
PY
