#!/usr/bin/env python3
"""Where do get_model's GPU witnesses lie?  The candidate cap
(model.SEARCH_CANDIDATES) bounds the device time a MISS costs before z3
decides the query; it should sit well above the first satisfying index of
the queries that do hit.

For every distinct stand-in query of the C1 / C3 / C4 / C5 streams
(mythril_amd/workloads.py) and the repository's own coupled-leaf / ABI test
queries, every dependence group is compiled as get_model compiles it and
searched with ``--cap`` candidates (batched per stream); the first index of
each hit is histogrammed.  Prints one JSON line per stream and a summary.

Usage: python tools/hit_index_census.py [--queries 512] [--cap 4194304]
"""

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

EDGES = (1, 16, 256, 4096, 1 << 16, 1 << 18, 1 << 20, 1 << 22)


def hist(idx):
    out = {}
    for e in EDGES:
        out["<%d" % e] = sum(i < e for i in idx)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queries", type=int, default=512)
    ap.add_argument("--cap", type=int, default=1 << 22)
    ap.add_argument("--streams", default="c1,c3,c4,c5")
    args = ap.parse_args()
    import mythril_amd.model as M
    from mythril_amd import workloads as W
    from mythril_amd.smt import symbol_factory
    BVV, BVS = symbol_factory.BitVecVal, symbol_factory.BitVecSym
    streams = {}
    for name in args.streams.split(","):
        seen, qs = set(), []
        for q in W.queries(name, 8 * args.queries):
            key = tuple(c.id for c in q)
            if key not in seen:
                seen.add(key)
                qs.append(M._raw_nodes(q))
            if len(qs) == args.queries:
                break
        streams[name] = qs
    # coupled constants in one group (tests/test_gpu_model.py)
    xs = [BVS("p%d" % i, 256) for i in range(4)]
    vals = [0x1234567, 0xDEADBEEF1, 0xABCDEF12345, 0x42424242]
    cs = [x == BVV(v, 256) for x, v in zip(xs, vals)] + [(xs[0] + xs[1] + xs[2] + xs[3]) != BVV(7, 256)]
    streams["tests"] = [M._raw_nodes(cs)]
    total = []
    for name, qs in streams.items():
        progs = []
        for nodes in qs:
            for b in M.dependence_buckets(nodes):
                try:
                    p = M._compile_search(b)
                except M.Unsupported:
                    continue
                if M._ground_value(p) is None:
                    progs.append(p)
        hits = M.batch_search_devices(progs, args.cap) if progs else []
        idx = [i for i, _ in hits if i >= 0]
        total += idx
        print(json.dumps({"stream": name, "queries": len(qs), "searched_groups": len(progs),
                          "hits": len(idx), "max_first_index": max(idx, default=-1),
                          "hist": hist(idx)}), flush=True)
    print(json.dumps({"summary": {"hits": len(total), "max_first_index": max(total, default=-1),
                                  "hist": hist(total), "cap": args.cap}}), flush=True)


if __name__ == "__main__":
    main()
