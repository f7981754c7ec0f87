"""The model construction refuses a commit that kills a satisfiable group
(round 6, solve.Solver.run / _culprit, mirrored in mg_compile.cpp): the C3
overflow checks after an approve (stream ``c3o``) used to compile to a
false root because two first-pass commits conflicted.  Now
the definition that completed the false root is refused and the
construction runs again, so the group is searched — here on the CPU, with
the device's leaf generator restated (``oracle/gen_ref.py``) and the
compiled program executed by ``tests/ir_sim.py``, until a candidate
satisfies it; the witness is then checked against the oracle on the source
query.  An UNSAT group stays without a witness (every original constraint
is evaluated), and the host refutation answers the SafeMath checks before
anything compiles."""

import numpy as np

import ir_sim
import mythril_amd.model as M
from mythril_amd import assign, workloads as W
from oracle import gen_ref as G
from oracle import smtlib_ref as R


def _limbs(vals):
    out = np.zeros((max(1, len(vals)), 8), dtype=np.uint32)
    for i, v in enumerate(vals):
        for k in range(8):
            out[i, k] = (v >> (32 * k)) & 0xFFFFFFFF
    return out


def _false_root(p):
    """A program that is its constant-false root (the dead-group form)."""
    return len(p.code) <= 2 and not ir_sim.run(p, [0] * len(p.leaves))[0]


def _first_witness(p, limit):
    gens = M.search_leafgen(p)
    for idx in range(limit):
        lv = [G.gen_leaf(M.SEARCH_SEED, 0, i, idx, g.width,
                         p.const_values[g.pool_off:g.pool_off + g.pool_n],
                         (g.pct_uniform, g.pct_small, g.pct_boundary))
              for i, g in enumerate(gens)]
        root, probes = ir_sim.run(p, lv)
        if root:
            return assign.unpack(p, _limbs(lv), _limbs(probes))
    return None


def test_overflow_check_after_an_approve_is_searched_and_solved():
    q = W.queries("c3o", 64)[16]
    parts = []
    for b in M.dependence_buckets(q):
        p = M._compile_search_uncached(b)
        assert not _false_root(p), "the group compiled to its false root"
        w = _first_witness(p, 4000)
        assert w is not None, "no candidate of 4000 satisfies the group"
        parts.append(w)
    w = M._merge(parts)
    assert R.eval_constraints(q, R.Assignment(w.vars, w.arrays, w.funcs)) == 1


def test_unsat_safemath_check_is_refuted_before_compiling_and_never_satisfied():
    """A refused commit can make a group that used to compile to its false
    root (an UNSAT SafeMath check) compile to a live program; it stays
    unsatisfiable (the program evaluates every original constraint), and
    get_model never compiles it: the host refutation answers it first."""
    from mythril_amd.refute import refuted
    qs = W.queries("c3", 64)
    q = next(q for q in qs if W.query_label(q).startswith("unsat: SafeMath.add"))
    groups = [b for b in M.dependence_buckets(q) if len(b) > 1]
    assert any(refuted(b) for b in groups)
    for b in groups:
        assert _first_witness(M._compile_search_uncached(b), 300) is None
