#!/usr/bin/env python3
"""Ground-truth labels for the stand-in query streams:
``tests/golden/recall_labels.json``.

For the first ``N`` queries of each stream (C1 / C3 / C4 / C5, the queries
tools/search_bench.py searches, and — round 6 — ``c3o``: the C3 stream's
batchTransfer overflow checks alone, SAT by construction, so C3's recall does
not rest on two queries):

* ``unsat`` — the stream generator labels the query UNSAT by construction
  (``workloads.query_label``: the SafeMath ``require`` on the same path that
  rules the check out, or — round 6 — the step at which a WalletLibrary
  path became infeasible: an m_pending entry nobody wrote, revoke's
  ownersDone, the never-written m_spentToday), or the host refutation
  proves it (``mythril_amd/refute.py``: exact per-pair order and interval
  reasoning, brute-force-checked in tests/test_refute.py; the reason names
  it).  As a cross-check the planter is still run on it with a small budget
  and must find nothing;
* ``sat`` — ``tests/planted.py`` found a model (ABI-aware scenarios + local
  search, independent of the engine's search) and ``oracle/smtlib_ref.py``
  accepts it; the model is stored, so tests/test_recall_labels.py re-checks
  it on every CPU run;
* ``unknown`` — neither.

Run in the build container (CPU only):  python tests/golden/make_recall_labels.py
"""

import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

N = 64
WORKLOADS = ("c1", "c3", "c4", "c5", "c3o")
OUT = os.path.join(HERE, "recall_labels.json")


def model_json(asg):
    return {"vars": {k: hex(v) for k, v in sorted(asg.vars.items())},
            "arrays": {k: [[hex(a), hex(b)] for a, b in t[0]] + [hex(t[1])]
                       for k, t in sorted(asg.arrays.items())},
            "funcs": {k: [[hex(a), hex(b)] for a, b in t[0]] + [hex(t[1])]
                      for k, t in sorted(asg.funcs.items())}}


def label_one(item):
    name, i = item
    import planted
    from mythril_amd import workloads as W
    q = W.queries(name, N)[i]
    why = W.query_label(q)
    if not why.startswith("unsat"):
        import mythril_amd.model as M
        from mythril_amd.refute import refuted
        if any(refuted(b) for b in M.dependence_buckets(q) if len(b) > 1):
            why = "unsat: refuted on the host (mythril_amd/refute.py: contradictory order / " \
                  "interval atoms)"
    if why.startswith("unsat"):
        asg = planted.plant(q, seed=i, restarts=2, steps=60)
        if asg is not None:
            raise SystemExit("%s query %d is labelled %r but a model satisfies it" % (name, i, why))
        return {"i": i, "label": "unsat", "why": why, "model": None}
    asg = planted.plant(q, seed=i, restarts=24, steps=300)
    return {"i": i, "label": "sat" if asg is not None else "unknown", "why": why,
            "model": model_json(asg) if asg is not None else None}


def main():
    from mythril_amd.procmap import process_map
    items = [(w, i) for w in WORKLOADS for i in range(N)]
    t0 = time.time()
    rows = process_map(label_one, items, min(8, os.cpu_count() or 1), "fork")
    out = {"n": N, "what": __doc__.split("\n\n")[0], "streams": {}}
    for (w, _), r in zip(items, rows):
        out["streams"].setdefault(w, []).append(r)
    for w, rs in out["streams"].items():
        print(w, {k: sum(r["label"] == k for r in rs) for k in ("sat", "unsat", "unknown")})
    with open(OUT, "w") as fh:
        json.dump(out, fh, indent=0, separators=(",", ":"))
    print("wrote %s in %.0f s" % (OUT, time.time() - t0))


if __name__ == "__main__":
    main()
