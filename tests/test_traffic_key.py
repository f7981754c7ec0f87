"""The committed HBM-traffic measurement (profiles/traffic.json) belongs to
the kernel this tree benchmarks.

bench.py reports ``roofline.traffic`` only when its kernel_key (generated
assembly, leaf policy, compiled-program code, workload and programs) equals
the key the FETCH_SIZE / WRITE_SIZE passes ran under; a kernel change that
is not followed by a fresh tools/profile.sh run would otherwise leave the
bench line with ``traffic: null``.  CPU-only: the key is computed from the
generator and the compiled corpus, no GPU."""
import json
import os

import bench
from mythril_amd import asmgen

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_traffic_json_keyed_to_this_tree():
    with open(os.path.join(ROOT, "profiles", "traffic.json")) as fh:
        tj = json.load(fh)
    entries = tj["entries"]
    corpus = bench.build_corpus(4096, min(8, os.cpu_count() or 1))
    key = bench.kernel_key(asmgen.digest(), "c2", 4096, 20, True, corpus)
    c2 = [e for e in entries if e["kernel_key"].get("workload") == "c2"]
    assert c2, "profiles/traffic.json has no C2 entry"
    diff = sorted(k for k in key if c2[0]["kernel_key"].get(k) != key[k])
    assert not diff, "profiles/traffic.json is for another kernel (%s differ): " \
        "re-run tools/profile.sh + tools/prof_summary.py" % ", ".join(diff)
    for e in entries:
        # FETCH doubled (gfx950 correction) + WRITE, KiB -> bytes
        assert e["hbm_bytes_per_launch"] == (2 * e["fetch_kib"] + e["write_kib"]) * 1024
    # one entry per (workload, size, path)
    slots = [(e["kernel_key"]["workload"], e["kernel_key"]["dags"], e["kernel_key"]["jit"])
             for e in entries]
    assert len(slots) == len(set(slots))
