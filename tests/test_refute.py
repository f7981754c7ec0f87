"""Host-side refutation (mythril_amd/refute.py): a group
whose atoms contradict each other is sent to z3 without a compile or a
launch.  The rule must never refute a satisfiable group (brute force over
small widths, every SAT-labelled stand-in query), must catch the SafeMath
shapes of the C3 stream, and the drop-in must then reach z3 without
concluding UNSAT itself."""

import itertools
import json
import os
import random

import pytest

import mythril_amd.model as M
from mythril_amd import workloads as W
from mythril_amd.refute import refuted
from mythril_amd.smt import (ULE, UGE, ULT, UGT, And, BVAddNoOverflow, BVMulNoOverflow, If, Not,
                             Or, symbol_factory)
from oracle import smtlib_ref as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
bv, sym = symbol_factory.BitVecVal, symbol_factory.BitVecSym


def raws(cs):
    return [c.raw for c in cs]


def test_pair_rules():
    x, y = sym("rx", 256), sym("ry", 256)
    assert refuted(raws([ULT(x, y), ULE(y, x)]))
    assert refuted(raws([UGE(x, y), ULT(x, y)]))              # LASER's UGE = Or(UGT, ==)
    assert refuted(raws([x == y, Not(x == y)]))
    assert refuted(raws([x == y, UGT(x, y)]))
    assert refuted(raws([x < y, y < x]))                       # signed
    assert not refuted(raws([x < y, UGT(x, y)]))               # signed and unsigned differ
    assert refuted(raws([x < y, x == y]))                      # equality is both
    assert not refuted(raws([ULT(x, y), ULT(y, sym("rz", 256))]))   # no transitivity claimed
    # LASER's JUMPI / ISZERO shape: If(c, 1, 0) == 0 is Not(c)
    jumpi = If(ULT(x, y), bv(1, 256), bv(0, 256)) == bv(0, 256)
    assert refuted(raws([jumpi, ULT(x, y)]))
    assert not refuted(raws([jumpi, ULE(x, y)]))


def test_intervals_and_overflow():
    x, y = sym("ix", 256), sym("iy", 256)
    assert refuted(raws([ULT(x, bv(5, 256)), UGT(x, bv(10, 256))]))
    assert refuted(raws([x == bv(3, 256), x == bv(4, 256)]))
    assert refuted(raws([x == bv(3, 256), Not(x == bv(3, 256))]))
    assert not refuted(raws([ULT(x, bv(5, 256)), UGT(x, bv(3, 256))]))
    # SafeMath.add: require(x + y >= x), then the carry of x + y
    s = x + y
    carry = Not(BVAddNoOverflow(x, y, False))
    assert refuted(raws([UGE(s, x), carry]))
    assert refuted(raws([UGE(y + x, y), carry]))               # either operand order
    assert not refuted(raws([carry]))
    assert not refuted(raws([UGE(s, x), BVAddNoOverflow(x, y, False)]))
    # batchTransfer's loop exit: cnt <= 1 cannot overflow cnt * value
    ovfl = Not(BVMulNoOverflow(x, y, False))
    assert refuted(raws([Not(ULT(bv(1, 256), x)), ovfl]))
    assert not refuted(raws([Not(ULT(bv(2, 256), x)), ovfl]))


def _random_formula(rng, xs, depth=2):
    """A conjunction over 4-bit terms from the rule's grammar and beyond it."""
    def term():
        k = rng.random()
        if k < 0.5:
            return rng.choice(xs)
        if k < 0.7:
            return bv(rng.choice([0, 1, 2, 7, 8, 12, 15, rng.randrange(16)]), 4)
        return rng.choice(xs) + rng.choice(xs)

    def atom():
        a, b = term(), term()
        op = rng.choice(["ult", "ule", "ugt", "uge", "slt", "sle", "eq"])
        f = {"ult": ULT, "ule": ULE, "ugt": UGT, "uge": UGE, "slt": lambda p, q: p < q,
             "sle": lambda p, q: p <= q, "eq": lambda p, q: p == q}[op](a, b)
        if rng.random() < 0.3:
            f = Not(f)
        if rng.random() < 0.2:
            f = If(f, bv(1, 4), bv(0, 4)) == bv(rng.choice([0, 1]), 4)
        return f

    cs = []
    for _ in range(rng.randrange(2, 6)):
        r = rng.random()
        if r < 0.2:
            cs.append(Or(atom(), atom()))
        elif r < 0.3:
            cs.append(And(atom(), atom()))
        else:
            cs.append(atom())
    return cs


def test_never_refutes_a_satisfiable_group_brute_force():
    """Random conjunctions over three 4-bit symbols (4096 assignments each,
    evaluated by the oracle): every refuted one has no model."""
    rng = random.Random(6)
    xs = [sym("bx", 4), sym("by", 4), sym("bz", 4)]
    n_ref = 0
    for _ in range(400):
        cs = _random_formula(rng, xs)
        if not refuted(raws(cs)):
            continue
        n_ref += 1
        nodes = raws(cs)
        for vx, vy, vz in itertools.product(range(16), range(16), range(16)):
            if R.eval_constraints(nodes, R.Assignment({"bx": vx, "by": vy, "bz": vz})):
                pytest.fail("refuted a satisfiable group: %d %d %d %r" % (vx, vy, vz, nodes))
    assert n_ref >= 20                     # the property was exercised


def test_stand_in_streams_sat_never_refuted_and_c3_unsat_refuted():
    with open(os.path.join(ROOT, "tests", "golden", "recall_labels.json")) as fh:
        labels = json.load(fh)["streams"]
    for name in ("c1", "c3", "c4", "c5"):
        lab = {r["i"]: r["label"] for r in labels[name]}
        qs = W.queries(name, 64)
        for i, q in enumerate(qs):
            ref = any(refuted(b) for b in M.dependence_buckets(q) if len(b) > 1)
            if lab.get(i) == "sat":
                assert not ref, (name, i)
            if name == "c3" and lab.get(i) == "unsat":
                assert ref, (name, i, W.query_label(q))


def test_refuted_query_goes_to_z3_without_compile_or_launch(monkeypatch):
    """get_model on a refuted query: no compile, no launch, the group is a
    miss at any depth, and the answer is z3's (here: z3 absent, so the
    engine never claims UNSAT — SolverUnavailable)."""
    monkeypatch.setattr(M.z3bridge, "available", lambda: False)
    M.get_model.cache_clear()
    M.clear_search_memos()
    M.args.solver_timeout = 10000
    M.time_handler.start_execution(3600)
    compiled, launched = [], []
    monkeypatch.setattr(M, "_compile_search", lambda b, *a: compiled.append(b))
    monkeypatch.setattr(M, "get_engine", lambda *a, **k: launched.append(a))
    x, y = sym("zx", 256), sym("zy", 256)
    q = (UGE(x, y), ULT(x, y))
    M.stats.reset_gpu()
    with pytest.raises(M.SolverUnavailable):
        M.get_model(q, enforce_execution_time=False)
    assert M.stats.refuted == 1 and not compiled and not launched
    key = M._group_key(M.dependence_buckets(M._raw_nodes(list(q)))[0])
    assert M._group_miss[key] == M.GROUND_MISS
    # with z3 "present", z3 is asked and its answer returned
    z3_calls = []

    def fake_z3(constraints, minimize, maximize, timeout):
        z3_calls.append(constraints)
        raise M.UnsatError
    monkeypatch.setattr(M, "_z3_check", fake_z3)
    monkeypatch.setattr(M.z3bridge, "available", lambda: True)
    M.get_model.cache_clear()
    with pytest.raises(M.UnsatError):
        M.get_model(q, enforce_execution_time=False)
    assert len(z3_calls) == 1 and not compiled and not launched
    # MYTHRIL_GPU_REFUTE=0 turns the rule off
    M.configure_from_env({"MYTHRIL_GPU_REFUTE": "0"})
    try:
        assert not M.REFUTE
    finally:
        M.configure_from_env({})
    assert M.REFUTE
    M.clear_search_memos()
    M.get_model.cache_clear()
