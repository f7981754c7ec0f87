#!/usr/bin/env python3
"""Does profiles/traffic.json describe the kernel this tree benchmarks?
Computes bench.py's kernel_key for the default configuration on the CPU
(programs compiled, library digest read; no GPU) and compares it with the
key the traffic measurement was taken under.  Exit 1 when they differ:
re-run tools/profile.sh on a GPU box before relying on roofline.traffic."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from mythril_amd.engine import load_library  # noqa: E402

corpus = bench.build_corpus(4096, min(8, os.cpu_count() or 1))
key = bench.kernel_key(load_library().mg_asm_digest().decode(), "c2", 4096, 20, True, corpus)
tj = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))
keys = [e["kernel_key"] for e in tj.get("entries", [])]
print(json.dumps({"tree": key, "traffic_json": keys, "match": key in keys}))
sys.exit(0 if key in keys else 1)
