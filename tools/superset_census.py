#!/usr/bin/env python3
"""Does the group-miss memo's SUPERSET rule lose GPU hits?  

``model._known_miss`` answers "miss" for a group that extends a group which
missed (LASER appends one JUMPI at a time), without searching it.  The new
constraint can define a leaf (``x == k``, solve.py definitions) and make the
model construction succeed where the subset's search failed; such a hit is
then lost to z3 (never an answer: z3 decides every miss).

For every stand-in stream (mythril_amd/workloads.py C1 / C3 / C4 / C5) the
distinct queries run through ``get_model`` in stream order with the memos
kept, exactly as LASER would ask them.  Every query the memo answered by the
superset rule is then searched anyway (SUPERSET_SKIP off, on a copy of the
memo state, so the stream itself is unchanged) and the outcome counted.

Prints one JSON line per stream and a summary.
Usage: python tools/superset_census.py [--queries 64]
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def distinct(name, n):
    from mythril_amd import workloads as W
    seen, out = set(), []
    for q in W.queries(name, 8 * n):
        key = tuple(c.id for c in q)
        if key not in seen:
            seen.add(key)
            out.append(q)
        if len(out) == n:
            break
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queries", type=int, default=64)
    ap.add_argument("--streams", default="c1,c3,c4,c5")
    args = ap.parse_args()
    import mythril_amd.model as M
    from mythril_amd.engine import get_engine
    get_engine(0)
    total = {"superset_answered": 0, "would_hit": 0}
    for name in args.streams.split(","):
        qs = distinct(name, args.queries)
        M.get_model.cache_clear()
        M.clear_search_memos()
        M.stats.reset_gpu()
        rows = []
        t0 = time.perf_counter()
        for i, q in enumerate(qs):
            nodes = M._raw_nodes(q)
            buckets = M.dependence_buckets(nodes)
            keys = [M._group_key(b) for b in buckets]
            exact = any(M._group_miss.get(k, -1) >= M.SEARCH_CANDIDATES for k in keys)
            superset = not exact and any(M._known_miss(k, M.SEARCH_CANDIDATES) for k in keys)
            probe = None
            if superset:
                # search it anyway, on a copy of the memo state
                saved = (dict(M._group_miss), {k: list(v) for k, v in M._miss_index.items()},
                         {k: list(v) for k, v in M._shape_stats.items()})
                M.SUPERSET_SKIP, M.SHAPE_GATE = False, False
                try:
                    hit = M.gpu_search(nodes, budget_ms=M.SEARCH_BUDGET_MS)
                    probe = hit is not None
                finally:
                    M.SUPERSET_SKIP, M.SHAPE_GATE = True, True
                    M._group_miss.clear()
                    M._group_miss.update(saved[0])
                    M._miss_index.clear()
                    M._miss_index.update(saved[1])
                    M._shape_stats.clear()
                    M._shape_stats.update(saved[2])
            before = M.stats.memo_misses
            M.get_model.cache_clear()
            try:
                M.get_model(tuple(q), enforce_execution_time=False)
                got = "hit"
            except M.SolverUnavailable:
                got = "miss"
            rows.append({"i": i, "groups": len(buckets), "memo": M.stats.memo_misses > before,
                         "superset": superset, "would_hit": probe, "result": got,
                         "newest": M.query_shape(nodes[-1]) if nodes else ""})
        sup = [r for r in rows if r["superset"]]
        line = {"stream": name, "queries": len(rows), "wall_s": time.perf_counter() - t0,
                "hits": sum(r["result"] == "hit" for r in rows),
                "memo_answered": sum(r["memo"] for r in rows),
                "superset_answered": len(sup),
                "superset_would_hit": sum(bool(r["would_hit"]) for r in sup),
                "would_hit_shapes": sorted({r["newest"] for r in sup if r["would_hit"]})}
        total["superset_answered"] += line["superset_answered"]
        total["would_hit"] += line["superset_would_hit"]
        print(json.dumps(line), flush=True)
    print(json.dumps({"summary": total}), flush=True)


if __name__ == "__main__":
    main()
