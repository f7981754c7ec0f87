#!/usr/bin/env python3
"""Which stand-in queries the batched search misses, by the shape of their
newest constraint (the module check / JUMPI a query is about): one batched
search per workload over its first N queries, as tools/search_bench.py
does, then the misses grouped by model.query_shape.
usage: tools/miss_census.py [workload] [n]"""
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import mythril_amd.model as M
    from mythril_amd import workloads as W
    from mythril_amd.engine import get_engine
    wl = sys.argv[1] if len(sys.argv) > 1 else "c4"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    eng = get_engine(0)
    qs = W.queries(wl, n)
    progs, qmap = [], []
    for qi, q in enumerate(qs):
        for b in M.dependence_buckets(q):
            progs.append(M._compile_search(b))
            qmap.append(qi)
    loaded = [eng.load(p, M.search_leafgen(p), prog_seed=0) for p in progs]
    hits = eng.batch_search(loaded, M.SEARCH_SEED, M.SEARCH_CANDIDATES)
    solved = [True] * len(qs)
    first = collections.defaultdict(list)
    for qi, (i, _), p in zip(qmap, hits, progs):
        solved[qi] = solved[qi] and i >= 0
        first[qi].append(i)
    census = collections.Counter()
    for qi, q in enumerate(qs):
        if not solved[qi]:
            census[M.query_shape(q[-1])] += 1
    idx = sorted(i for v in first.values() for i in v if i >= 0)
    print(json.dumps({"workload": wl, "queries": n, "hits": sum(solved),
                      "first_index_median": idx[len(idx) // 2] if idx else None,
                      "first_index_max": idx[-1] if idx else None,
                      "missed_by_shape": census.most_common()}, indent=1))


if __name__ == "__main__":
    main()
