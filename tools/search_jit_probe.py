#!/usr/bin/env python3
"""Would compiled programs pay on the get_model search path?  (VERDICT r3
item 4: the search runs the record interpreter.)

For distinct stand-in queries of a stream, each independent group's search
program (model._compile_search_uncached, as get_model compiles it) is run
three ways on one GPU context:

* interpreter: ``Engine.search`` over the query's candidate budget;
* compiled: the same program with its straight-line code attached
  (jit.compile_batch of that one program, then ``mg_jit_attach``);

and the cost of getting the code there: the host assembly time
(``compile_batch``) and the attach time (``hipModuleLoadData`` + table
read + descriptor patch).  The first index and witness must agree.

Prints one JSON line per stream.  Usage: tools/search_jit_probe.py
[--stream c3] [--queries 16]
"""

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", default="c1,c3,c4")
    ap.add_argument("--queries", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import mythril_amd.model as M
    from mythril_amd import jit
    from mythril_amd import workloads as W
    from mythril_amd.engine import get_engine
    eng = get_engine(0)
    for name in args.streams.split(","):
        seen, progs = set(), []
        for q in W.queries(name, 8 * args.queries):
            key = tuple(c.id for c in q)
            if key in seen:
                continue
            seen.add(key)
            for b in M.dependence_buckets(M._raw_nodes(q)):
                try:
                    progs.append(M._compile_search_uncached(b))
                except M.Unsupported:
                    pass
            if len(seen) >= args.queries:
                break
        rows = []
        for p in progs:
            n_cand = M._n_cand([p], M.SEARCH_BUDGET_MS)
            lg = M.search_leafgen(p)
            t0 = time.perf_counter()
            try:
                image = jit.compile_batch([(p, lg, 0)])
            except Exception as e:       # noqa: BLE001 - reported, not fatal
                rows.append({"ins": int(p.n_ins), "error": "%s: %s" % (type(e).__name__, e)})
                continue
            t_asm = time.perf_counter() - t0
            lp = eng.load(p, lg, prog_seed=0)
            ti = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                r_i = eng.search(lp, M.SEARCH_SEED, n_cand)
                ti.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            h = eng.jit_attach([lp], image)
            t_att = time.perf_counter() - t0
            tj = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                r_j = eng.search(lp, M.SEARCH_SEED, n_cand)
                tj.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            eng.jit_detach(h)
            t_det = time.perf_counter() - t0
            same = r_i[0] == r_j[0] and (r_i[1] is None or (r_i[1] == r_j[1]).all())
            rows.append({"ins": int(p.n_ins), "n_cand": n_cand, "first": r_i[0], "same": bool(same),
                         "interp_ms": min(ti) * 1e3, "jit_ms": min(tj) * 1e3,
                         "asm_ms": t_asm * 1e3, "attach_ms": t_att * 1e3, "detach_ms": t_det * 1e3,
                         "image_kb": len(image) / 1024})
        ok = [r for r in rows if "error" not in r]
        med = lambda k: statistics.median(r[k] for r in ok) if ok else None  # noqa: E731
        print(json.dumps({"stream": name, "programs": len(rows), "errors": len(rows) - len(ok),
                          "all_same": all(r["same"] for r in ok),
                          "median": {k: med(k) for k in ("ins", "interp_ms", "jit_ms", "asm_ms",
                                                         "attach_ms", "detach_ms", "image_kb")},
                          "sum_interp_ms": sum(r["interp_ms"] for r in ok),
                          "sum_jit_ms": sum(r["jit_ms"] for r in ok),
                          "sum_attach_ms": sum(r["attach_ms"] for r in ok),
                          "rows": rows}), flush=True)


if __name__ == "__main__":
    main()
