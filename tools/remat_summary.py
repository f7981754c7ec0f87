#!/usr/bin/env python3
"""Summarise tools/ab_leaf_remat.sh output (gpurun_out/remat): per leaf
eviction policy, the bench value / kernel time and the HBM bytes per
mg_interp dispatch (FETCH_SIZE doubled per the gfx950 correction + WRITE_SIZE,
as tools/prof_summary.py).  Writes profiles/<round>/leaf_remat_ab.json."""
import csv
import glob
import json
import os
import sys

ROUND = sys.argv[1] if len(sys.argv) > 1 else "r02"
SRC = "gpurun_out/remat"


def pmc(pol, kind, counter):
    f = glob.glob(os.path.join(SRC, "%s_%s" % (kind, pol), "**", "*counter_collection.csv"),
                  recursive=True)
    if not f:
        return None
    tot = {}
    for r in csv.DictReader(open(f[0])):
        if "mg_interp" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            tot[r["Dispatch_Id"]] = tot.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return max(tot.values()) if tot else None


out = {}
for log in sorted(glob.glob(os.path.join(SRC, "bench_*.log"))):
    pol = os.path.basename(log)[len("bench_"):-len(".log")]
    t = open(log).read()
    d = json.loads(t[t.index("{"):].splitlines()[0])
    fetch, write = pmc(pol, "fetch", "FETCH_SIZE"), pmc(pol, "write", "WRITE_SIZE")
    out[pol] = {"value_G": d["value"] / 1e9, "frac": d["roofline"]["frac"],
                "kernel_ms": d["roofline"]["kernel_ms"],
                "fetch_kib": fetch, "write_kib": write,
                "hbm_TB_per_launch": None if fetch is None or write is None
                else (2 * fetch + write) * 1024 / 1e12}
    print(pol, json.dumps(out[pol]))
os.makedirs(os.path.join("profiles", ROUND), exist_ok=True)
json.dump(out, open(os.path.join("profiles", ROUND, "leaf_remat_ab.json"), "w"), indent=1)
