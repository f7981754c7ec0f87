#!/bin/bash
# Where a workload's wave time goes (round 6): two SQ counter passes of the
# default compiled-program bench configuration (<= 8 SQ counters + GRBM each),
# the images prebuilt outside the profiler.
# usage: tools/prof_stalls_w.sh <tag> [bench args...]
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
TAG=$1; shift
P=gpurun_out/stalls_$TAG
mkdir -p $P
export MYTHGPU_JIT_CACHE=/tmp/mg_jitcache
export MYTHGPU_BENCH_WORKERS=1
( while true; do date >> $P/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
ARGS="--steps 1 --warmup 0 --no-cpu-baseline $@"
MYTHGPU_BENCH_WORKERS=16 timeout -k 10 600 python3 bench.py --jit-build-only $@ > $P/prebuild.log 2>&1 || { tail -5 $P/prebuild.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --output-format csv -d $P/st1 -o st1 -- python3 bench.py $ARGS > $P/st1.log 2>&1 || { tail -5 $P/st1.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d $P/st2 -o st2 -- python3 bench.py $ARGS > $P/st2.log 2>&1 || { tail -5 $P/st2.log; exit 1; }
python3 - $P <<'PY'
import csv, glob, json, sys
P = sys.argv[1]
c = {}
for f in glob.glob(P + "/st*/**/*counter_collection.csv", recursive=True):
    per = {}
    for r in csv.DictReader(open(f)):
        if "mg_interp_asm<0>" in r["Kernel_Name"]:
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    # the dominant (largest-wave) dispatch of each pass
    disp = {}
    for (d, n), v in per.items():
        disp.setdefault(d, {})[n] = v
    best = max(disp.values(), key=lambda m: m.get("SQ_WAVES", m.get("SQ_INSTS_VALU", 0)))
    c.update(best)
w = c.get("SQ_WAVES", 1.0)
out = {k: v for k, v in sorted(c.items())}
out["per_wave"] = {k: v / w for k, v in sorted(c.items()) if k not in ("SQ_WAVES", "GRBM_GUI_ACTIVE")}
wc = c.get("SQ_WAVE_CYCLES", 0) or 1
out["share_of_wave_cycles"] = {k: c[k] / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                      "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA",
                                                      "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS") if k in c}
print(json.dumps(out, indent=1))
json.dump(out, open(P + "/stalls.json", "w"), indent=1)
PY
echo stalls-ok
