"""The ground-truth labels of the stand-in streams (VERDICT r4 item 4,
``tests/golden/recall_labels.json``, made by
``tests/golden/make_recall_labels.py``) stay true: every planted model of a
SAT-labelled query is accepted by the oracle, every UNSAT label is the
generator's own (a SafeMath require on the path, or the step at which a
WalletLibrary path became infeasible) or a host refutation
(mythril_amd/refute.py, whose soundness tests/test_refute.py checks by brute
force), and the streams the labels index are the streams the code
generates."""

import json
import os

import pytest

from mythril_amd import workloads as W
from oracle import smtlib_ref as R

HERE = os.path.dirname(os.path.abspath(__file__))
LABELS = json.load(open(os.path.join(HERE, "golden", "recall_labels.json")))


def assignment(m):
    def table(t):
        return ([(int(a, 16), int(b, 16)) for a, b in t[:-1]], int(t[-1], 16))
    return R.Assignment({k: int(v, 16) for k, v in m["vars"].items()},
                        {k: table(t) for k, t in m["arrays"].items()},
                        {k: table(t) for k, t in m["funcs"].items()})


@pytest.mark.parametrize("stream", sorted(LABELS["streams"]))
def test_planted_models_satisfy_their_queries(stream):
    qs = W.queries(stream, LABELS["n"])
    rows = LABELS["streams"][stream]
    assert [r["i"] for r in rows] == list(range(LABELS["n"]))
    for r in rows:
        q = qs[r["i"]]
        if r["why"].startswith("unsat: refuted on the host"):
            # the generator claims nothing; the host refutation proves it
            import mythril_amd.model as M
            from mythril_amd.refute import refuted
            assert not W.query_label(q).startswith("unsat"), r["i"]
            assert any(refuted(b) for b in M.dependence_buckets(q) if len(b) > 1), r["i"]
        else:
            assert r["why"] == W.query_label(q), r["i"]
        if r["label"] == "sat":
            assert R.eval_constraints(q, assignment(r["model"])) == 1, (stream, r["i"])
        elif r["label"] == "unsat":
            assert r["why"].startswith("unsat:") and r["model"] is None
        else:
            assert r["label"] == "unknown" and r["model"] is None


def test_every_stream_has_sat_and_the_overflow_streams_unsat_labels():
    count = {s: {k: sum(r["label"] == k for r in rows) for k in ("sat", "unsat", "unknown")}
             for s, rows in LABELS["streams"].items()}
    assert all(c["sat"] > 0 for c in count.values()), count
    assert count["c3"]["unsat"] > 0, count


def test_no_sat_labelled_group_compiles_to_its_false_root():
    """The model construction never kills a satisfiable group (round 6:
    refused commits, solve.Solver.run): for every SAT-labelled query, no
    independent group compiles to its constant-false root (13 c3o groups
    and C5 query 52 did before)."""
    import mythril_amd.model as M
    dead = []
    for stream, rows in LABELS["streams"].items():
        qs = W.queries(stream, LABELS["n"])
        for r in rows:
            if r["label"] != "sat":
                continue
            for b in M.dependence_buckets(qs[r["i"]]):
                if len(b) < 2:
                    continue
                if M._ground_value(M._compile_search_uncached(b)) is False:
                    dead.append((stream, r["i"]))
    assert not dead, dead
