"""Algorithmic work weights (mythril_amd/roofline.py) — round 5
(VERDICT r4 item 1): work the lowering does by a cheaper algorithm than its
operator's generic weight is priced at that algorithm's cost, so a
workload's weighted ops never exceed what the kernel must execute."""

import numpy as np
import pytest

import bench
from mythril_amd import irdefs as I
from mythril_amd.ir import compile_constraints
from mythril_amd.roofline import calldata_word, dag_work, node_weight
from mythril_amd.smt import node as N
from mythril_amd.smt.node import topo_order


def _w(n, ts=None):
    return dag_work([N.bv_cmp("bvult", n, N.bv_var("z", n.width))], ts)[1] - 8.0 * (n.width // 32) / 8


x = N.bv_var("x", 256)
y = N.bv_var("y", 256)


@pytest.mark.parametrize("k", [0, 1, 5, 64, 255])
@pytest.mark.parametrize("op", ["bvudiv", "bvurem"])
def test_division_by_a_power_of_two_weighs_an_extract(op, k):
    q = N.bv_op(op, x, N.bv_num(1 << k, 256))
    assert _w(q) == node_weight(N.extract(200, 0, x), {}) == 8.0


@pytest.mark.parametrize("op", ["bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod"])
def test_general_division_keeps_its_weight(op):
    assert _w(N.bv_op(op, x, N.bv_num(6, 256))) == 512.0
    assert _w(N.bv_op(op, x, y)) == 512.0
    # signed division by 2^k is not a plain bit-field op (rounding toward 0)
    if op == "bvsdiv":
        assert _w(N.bv_op(op, x, N.bv_num(8, 256))) == 512.0


@pytest.mark.parametrize("op", ["bvshl", "bvlshr", "bvashr"])
def test_constant_shift_weighs_a_bitfield_move(op):
    assert _w(N.bv_op(op, x, N.bv_num(17, 256))) == 8.0
    assert _w(N.bv_op(op, x, y)) == 24.0


def _word(cd, off, size, *, skip=None):
    """LASER's calldata word (calldata.py:47-54,219-232)."""
    terms = []
    for i in range(32):
        idx = off if i == 0 else N.bv_op("bvadd", off, N.bv_num(i, 256))
        t = N.ite(N.bv_cmp("bvslt", idx, size), N.select(cd, idx), N.bv_num(0, 8))
        terms.append(t)
    return N.concat(*terms), terms


def test_calldata_word_is_one_lookup():
    cd = N.array_var("1_calldata", 256, 8)
    off, size = N.bv_var("off", 256), N.bv_var("1_calldatasize", 256)
    w, terms = _word(cd, off, size)
    assert calldata_word(w) is not None
    for E in (1, 2, 5):
        nodes, weight = dag_work([N.bv_cmp("bvult", w, y)], {"1_calldata": E})
        # the word (16 E + 24) and the ult (8); every byte term absorbed, but
        # every node still counted (the metric's unit)
        assert weight == 16 * E + 24 + 8
        assert nodes == 1 + 1 + 32 * 3 + 31
    # a byte term read outside the word keeps its weight (and its compare,
    # select and index): the lowering computes it for that reader
    other = N.bv_cmp("bvult", N.zero_extend(248, terms[5]), y)
    _, w2 = dag_work([N.bv_cmp("bvult", w, y), other], {"1_calldata": 2})
    sel = node_weight(terms[5].args[1], {"1_calldata": 2})
    # word + its ult; the other ult, zero_extend, ite, slt, select, index add
    assert w2 == (16 * 2 + 24 + 8) + 8 + 8 + (1 + 8 + sel + 8)


def test_words_recognised_equal_fused_words_compiled():
    """The roofline's recogniser prices exactly the words the lowering fuses:
    per unit, recognised words == CDWX instructions of the eval program."""
    for wl, ids in (("c3", range(0, 64, 4)), ("c4", range(0, 64, 4)), ("c5", range(0, 128, 8))):
        for d in ids:
            roots = bench.workload_roots(wl, d)
            prog = compile_constraints(roots)
            words = sum(calldata_word(n) is not None for n in topo_order(list(roots)))
            assert words == int(np.sum((prog.code[:, 0] & 0xFF) == I.CDWX)), (wl, d)


def test_c2_weights_unchanged_by_the_new_rules():
    """C2's corpus has no constant shifts, power-of-two divisors or calldata
    words: its weights (the headline roofline) are those of round 4."""
    from mythril_amd.corpus import make_dag
    for d in range(0, 4096, 512):
        roots = make_dag(d, bench.SEED)[0]
        order = topo_order(list(roots))
        assert not any(calldata_word(n) for n in order)
