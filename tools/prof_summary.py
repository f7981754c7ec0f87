#!/usr/bin/env python3
"""Summarise gpurun_out/prof[_<tag>] into profiles/<round>/[<tag>/] and
profiles/traffic.json (HBM traffic and, since round 5, the SQ pass of the same
kernel: bench.py reports both only for the kernel_key they were measured on).

usage: tools/prof_summary.py <round> [<tag>]   (tag: the workload profiled
by ``PROF_TAG=<tag> tools/profile.sh --workload <tag>``; none = the default
C2 bench).  traffic.json holds one entry per kernel_key: a new measurement
replaces the entry of the same workload / size / code path."""
import csv
import glob
import json
import os
import shutil
import sys

ROUND = sys.argv[1] if len(sys.argv) > 1 else "r01"
TAG = sys.argv[2] if len(sys.argv) > 2 else ""
SRC = "gpurun_out/prof" + ("_" + TAG if TAG else "")
DST = os.path.join("profiles", ROUND, TAG) if TAG else os.path.join("profiles", ROUND)
os.makedirs(DST, exist_ok=True)


def find(pat):
    f = glob.glob(os.path.join(SRC, pat), recursive=True)
    return f[0] if f else None


stats = find("kt/**/*kernel_stats.csv")
if stats:
    shutil.copy(stats, os.path.join(DST, "kernel_stats.csv"))
    for r in csv.DictReader(open(stats)):
        print("kernel", r.get("Name", "")[:60], "calls", r.get("Calls"), "avg_ns", r.get("AverageNs"))


def pmc(pat, counter):
    f = find(pat)
    if not f:
        return None
    tot = {}
    for r in csv.DictReader(open(f)):
        if "mg_interp" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            tot[r["Dispatch_Id"]] = tot.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    shutil.copy(f, os.path.join(DST, os.path.basename(os.path.dirname(f)) + "_" + counter + ".csv"))
    return max(tot.values()) if tot else None


def bench_line(log):
    """The JSON line bench.py printed in a profiled run (its kernel_key says
    which kernel the counters belong to)."""
    try:
        for line in open(os.path.join(SRC, log)):
            if line.startswith("{"):
                return json.loads(line)
    except OSError:
        pass
    return None


SIMDS = 256 * 4            # MI355X: 256 CUs x 4 SIMDs
N_XCD = 8


def sq_summary(path):
    """SQ / GRBM counters of the dominant mg_interp dispatch of the SQ pass
    (the bench launch; the handler-offset query launch is tiny), and what
    they say per launch:
      valu_insts      — SQ_INSTS_VALU, wave64 VALU instructions issued;
      valu_active     — share of the SIMDs' cycles with a VALU instruction
                        issuing: SQ_ACTIVE_INST_VALU counts quad-cycles
                        (MI355X_MICROARCH.md), summed over waves, against
                        GRBM_GUI_ACTIVE / 8 kernel cycles x 1024 SIMDs;
      valu_active_per_wave — SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (times the
                        resident waves per SIMD this is the same share when
                        the SIMDs stay full)."""
    per = {}
    for r in csv.DictReader(open(path)):
        if "mg_interp" in r["Kernel_Name"]:
            d = per.setdefault(r["Dispatch_Id"], {})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    if not per:
        return None
    c = max(per.values(), key=lambda d: d.get("SQ_WAVE_CYCLES", 0.0))
    w = c.get("SQ_WAVES") or 1.0
    summ = {k: c[k] for k in sorted(c)}
    summ.update({"dispatches": len(per),
                 "valu_insts": c.get("SQ_INSTS_VALU", 0.0),
                 "valu_per_wave": c.get("SQ_INSTS_VALU", 0) / w,
                 "salu_per_wave": c.get("SQ_INSTS_SALU", 0) / w,
                 "smem_per_wave": c.get("SQ_INSTS_SMEM", 0) / w,
                 "note": "the dominant mg_interp dispatch of the SQ pass (same bench "
                         "configuration as the traffic passes); SQ_WAVE_CYCLES / SQ_WAIT_* / "
                         "SQ_ACTIVE_INST_* count quad-cycles"})
    if c.get("SQ_WAVE_CYCLES"):
        summ["valu_active_per_wave"] = c.get("SQ_ACTIVE_INST_VALU", 0) / c["SQ_WAVE_CYCLES"]
        summ["salu_active_per_wave"] = c.get("SQ_ACTIVE_INST_SALU", 0) / c["SQ_WAVE_CYCLES"]
        summ["wait_inst_per_wave"] = c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
    if c.get("GRBM_GUI_ACTIVE"):
        cycles = c["GRBM_GUI_ACTIVE"] / N_XCD
        summ["kernel_cycles"] = cycles
        summ["valu_active"] = 4.0 * c.get("SQ_ACTIVE_INST_VALU", 0) / (cycles * SIMDS)
    return summ


fetch_kb = pmc("fetch/**/*counter_collection.csv", "FETCH_SIZE")
write_kb = pmc("write/**/*counter_collection.csv", "WRITE_SIZE")
sq = find("sq/**/*counter_collection.csv")
for log in glob.glob(os.path.join(SRC, "*.log")):
    shutil.copy(log, os.path.join(DST, os.path.basename(log)))
summ = None
if sq:
    shutil.copy(sq, os.path.join(DST, "sq_counters.csv"))
    summ = sq_summary(sq)
    if summ is not None:
        summ["kernel_key"] = (bench_line("sq.log") or {}).get("kernel_key")
        json.dump(summ, open(os.path.join(DST, "sq_summary.json"), "w"), indent=1)
        print("sq", json.dumps(summ))
if fetch_kb is not None and write_kb is not None:
    # FETCH_SIZE / WRITE_SIZE are in KiB per dispatch; gfx950 FETCH_SIZE counts
    # wide streaming reads at half their bytes (MI355X_MICROARCH.md §HBM):
    # report both the raw sum and the read-doubled upper bound.
    raw = (fetch_kb + write_kb) * 1024
    doubled = (2 * fetch_kb + write_kb) * 1024
    keys = [(bench_line(l) or {}).get("kernel_key") for l in ("fetch.log", "write.log")]
    if keys[0] != keys[1] or keys[0] is None:
        sys.exit("FETCH and WRITE passes ran different kernels: %s" % keys)
    out = {"kernel_key": keys[0], "fetch_kib": fetch_kb, "write_kib": write_kb,
           "hbm_bytes_per_launch": doubled, "hbm_bytes_raw": raw, "round": ROUND,
           "evidence": DST,
           "note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, per mg_interp "
                   "dispatch of this bench config; read side doubled per the gfx950 "
                   "FETCH_SIZE correction (upper bound)"}
    if summ is not None:
        if summ.get("kernel_key") != keys[0]:
            sys.exit("the SQ pass ran another kernel than the traffic passes: %s vs %s"
                     % (summ.get("kernel_key"), keys[0]))
        out["sq"] = {k: summ[k] for k in ("valu_insts", "valu_per_wave", "valu_active",
                                          "valu_active_per_wave", "kernel_cycles",
                                          "SQ_WAVES") if k in summ}
    path = "profiles/traffic.json"
    try:
        tj = json.load(open(path))
    except (OSError, ValueError):
        tj = {}
    entries = tj.get("entries", [tj] if "kernel_key" in tj else [])

    def slot(k):
        return (k.get("workload"), k.get("dags"), k.get("assign_log2"), k.get("jit"))
    entries = [e for e in entries if slot(e["kernel_key"]) != slot(out["kernel_key"])] + [out]
    json.dump({"entries": entries}, open(path, "w"), indent=1)
    print("traffic", out)
