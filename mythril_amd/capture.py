"""Capture and replay of ``get_model`` queries.

Capture (on a machine that runs Mythril with z3)::

    from mythril_amd import capture
    capture.install("queries.jsonl")     # after mythril_amd.model.install()
    ... myth analyze ...

wraps the ``get_model`` that Mythril calls (all three bindings, SURVEY.md
§8b) and appends one JSON line per call: the constraints as SMT-LIB 2
(:func:`mythril_amd.smtlib.dump_query`, z3 ASTs flattened through
:mod:`mythril_amd.z3bridge`), whether minimize/maximize were given, the
outcome (``sat`` / ``unsat`` / the exception name), the wall time and the
GPU pre-filter counters it moved.  These files are the C1/C3/C4 corpora of
SURVEY.md §8d.

Replay (here, or on the GPU box)::

    python -m mythril_amd.capture replay queries.jsonl [--gpu]

parses every query back, compiles it for the engine and reports the
operator census (which z3 operators occur, which the IR does not lower), and
with ``--gpu`` searches every optimisation-free query in one batched search
(:func:`mythril_amd.model.batch_is_possible` machinery).  A GPU witness for a
query recorded as ``unsat`` is a soundness bug and is reported as such.
"""

from __future__ import annotations

import argparse
import collections
import json
import sys
import time
from typing import Dict, List, Optional

from . import smtlib
from .smt import node as N

_installed: Optional[dict] = None


def _nodes(constraints) -> List[N.Node]:
    from . import model as M
    return M._raw_nodes([c for c in constraints if type(c) != bool])


class Recorder:
    """Wraps a ``get_model`` implementation and logs every call."""

    def __init__(self, path: str, inner):
        self.path = path
        self.inner = inner
        self.n = 0

    def __call__(self, constraints, minimize=(), maximize=(), enforce_execution_time=True):
        from . import model as M
        rec = {"id": self.n, "minimize": len(minimize), "maximize": len(maximize),
               "python_bools": [c for c in constraints if type(c) == bool]}
        self.n += 1
        try:
            rec["smt2"] = smtlib.dump_query(_nodes(constraints))
        except Exception as e:                  # unsupported z3 operator, ...
            rec["smt2"] = None
            rec["dump_error"] = "%s: %s" % (type(e).__name__, e)
        before = (M.stats.gpu_queries, M.stats.gpu_hits, M.stats.fallbacks)
        t0 = time.perf_counter()
        try:
            out = self.inner(constraints, minimize, maximize, enforce_execution_time)
            rec["result"] = "sat"
            return out
        except Exception as e:
            rec["result"] = "unsat" if type(e).__name__ == "UnsatError" else type(e).__name__
            raise
        finally:
            rec["ms"] = (time.perf_counter() - t0) * 1e3
            after = (M.stats.gpu_queries, M.stats.gpu_hits, M.stats.fallbacks)
            rec["gpu_queries"], rec["gpu_hits"], rec["fallbacks"] = [
                a - b for a, b in zip(after, before)]
            with open(self.path, "a") as fh:
                fh.write(json.dumps(rec) + "\n")


def install(path: str, modules=("mythril.support.model", "mythril.analysis.solver",
                                "mythril.laser.ethereum.state.constraints")) -> Recorder:
    """Log every ``get_model`` call of a Mythril installation to ``path``.
    The recorder wraps whatever those modules bind now (stock or GPU)."""
    import importlib
    global _installed
    mods = [importlib.import_module(m) for m in modules]
    rec = Recorder(path, mods[0].get_model)
    _installed = {m: m.get_model for m in mods}
    for m in mods:
        m.get_model = rec
    return rec


def uninstall() -> None:
    global _installed
    if _installed:
        for m, f in _installed.items():
            m.get_model = f
    _installed = None


def read(path: str) -> List[dict]:
    with open(path) as fh:
        return [json.loads(line) for line in fh if line.strip()]


def census(records: List[dict]) -> Dict[str, object]:
    """Operator counts over the captured queries and the queries the IR
    cannot lower (Unsupported), by reason."""
    from .ir import Unsupported, compile_constraints
    ops: collections.Counter = collections.Counter()
    unsupported: collections.Counter = collections.Counter()
    nodes = compiled = 0
    for r in records:
        if not r.get("smt2"):
            unsupported["not captured: " + r.get("dump_error", "?")] += 1
            continue
        cs = smtlib.parse_query(r["smt2"])
        for n in N.topo_order(cs):
            ops[n.op] += 1
            nodes += 1
        try:
            compile_constraints(cs)
            compiled += 1
        except Unsupported as e:
            unsupported[str(e)] += 1
    return {"queries": len(records), "nodes": nodes, "compiled": compiled,
            "ops": dict(ops.most_common()), "unsupported": dict(unsupported)}


def replay_gpu(records: List[dict]) -> Dict[str, object]:
    """Batched GPU search over the optimisation-free captured queries;
    compares with the recorded outcomes.  ``witnesses`` maps a query id to
    the joint model the GPU found (its groups' witnesses merged)."""
    from . import model as M
    from .ir import Unsupported
    sets, idx = [], []
    for r in records:
        if r.get("smt2") and not r["minimize"] and not r["maximize"] \
                and not any(b is False for b in r.get("python_bools", [])):
            try:
                cs = smtlib.parse_query(r["smt2"])
                M.dependence_buckets(cs)
            except (smtlib.ParseError, Unsupported):
                continue
            sets.append(cs)
            idx.append(r["id"])
    per_set, owner = [], []
    for k, cs in enumerate(sets):
        try:            # all of a set's groups or none (a partial set is no witness)
            per_set.append([M._compile_search(b) for b in M.dependence_buckets(cs)])
        except Unsupported:
            continue
        owner += [k] * len(per_set[-1])
    t0 = time.perf_counter()
    # (index, model) per group, one batched search; constant groups on the host
    hits = M._search_sets(per_set, M.SEARCH_CANDIDATES)
    secs = time.perf_counter() - t0
    found = collections.defaultdict(list)
    for k, (i, a) in zip(owner, hits):
        found[k].append(a if i >= 0 else None)
    by_id = {r["id"]: r for r in records}
    out = {"searched": len(sets), "gpu_found": 0, "seconds": secs, "unsound": [],
           "witnesses": {}}
    for k, qid in enumerate(idx):
        if found.get(k) and all(a is not None for a in found[k]):
            out["gpu_found"] += 1
            out["witnesses"][qid] = M._merge(found[k])      # the joint model
            if by_id[qid]["result"] == "unsat":
                out["unsound"].append(qid)
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m mythril_amd.capture")
    sub = ap.add_subparsers(dest="cmd", required=True)
    rp = sub.add_parser("replay", help="census (and GPU search) of a captured query file")
    rp.add_argument("path")
    rp.add_argument("--gpu", action="store_true")
    args = ap.parse_args(argv)
    records = read(args.path)
    report = {"census": census(records)}
    if args.gpu:
        report["gpu"] = replay_gpu(records)
        report["gpu"]["witnesses"] = {str(k): {"vars": {n: hex(v) for n, v in a.vars.items()}}
                                      for k, a in report["gpu"]["witnesses"].items()}
    print(json.dumps(report, indent=1))
    return 1 if report.get("gpu", {}).get("unsound") else 0


if __name__ == "__main__":
    sys.exit(main())
