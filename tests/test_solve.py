"""Search-mode model construction (mythril_amd/solve.py) on the query shapes
LASER builds: each rule turns a constraint random guessing cannot meet into a
definition, and every candidate's model — generated leaves plus the values
the program computed — gets the oracle's verdict on the ORIGINAL query equal
to the program's root bit (definitions never make the search unsound)."""

import numpy as np
import pytest

import ir_sim
from mythril_amd import workloads as W
from mythril_amd.assign import unpack
from mythril_amd.ir import compile_constraints
from mythril_amd.smt import node as N
from oracle import gen_ref
from oracle import smtlib_ref as R


def _pack1(vals):
    return np.array([[(v >> (32 * j)) & 0xFFFFFFFF for j in range(8)] for v in vals],
                    dtype=np.uint32).reshape(-1, 8)


def search(q, n=128, seed=11):
    """(program, hits): every candidate's root bit checked against the oracle
    on the unpacked model."""
    prog = compile_constraints(q, const_keys=True, leaf_pools=True, solve=True)
    table = [sum(int(prog.consts[i, j]) << (32 * j) for j in range(8))
             for i in range(prog.consts.shape[0])]
    hits = 0
    for idx in range(n):
        lv = []
        for li, l in enumerate(prog.leaves):
            off, cnt = prog.pool_ranges[li]
            lv.append(gen_ref.gen_leaf(seed, 0, li, idx, l.width, table[off:off + cnt],
                                       pct=(20, 40, 60)))
        root, probes = ir_sim.run(prog, lv)
        a = unpack(prog, _pack1(lv), _pack1(probes))
        assert root == R.eval_constraints(q, R.Assignment(a.vars, a.arrays, a.funcs)), idx
        hits += root
    return prog, hits


def defined(prog):
    return {prog.leaves[li].name for li in prog.derived}


def test_selector_bytes_are_defined():
    """``0xffffffff & calldata.word(0) / 2^224 == sel`` (the dispatcher)
    pins calldata[0..3] through udiv-by-2^k, the mask, the byte concat and
    the ``i < calldatasize`` guards."""
    w = W.World()
    t = w.tx()
    t.dispatch([0x18160DDD, 0xA9059CBB], 1)
    prog, hits = search(w.query())
    assert {"0_calldata#c%d#0" % i for i in range(4)} <= defined(prog)
    assert hits > 0


def test_actor_domain_becomes_a_selector():
    """``sender = A or sender = B or sender = C`` (symbolic.py's actor Or)."""
    w = W.World()
    w.tx()
    prog, hits = search(w.query())
    assert "sender_0" in defined(prog)
    assert any(l.kind == "aux" for l in prog.leaves)
    assert hits > 32                      # balance >= callvalue is the only guess left


def test_ite_flag_constraints():
    """``ite(c, 1, 0) != 0`` / ``= 0`` (ISZERO then JUMPI) reduce to ``c`` /
    ``not c``: nonpayable pins callvalue = 0."""
    w = W.World()
    t = w.tx()
    t.nonpayable()
    prog, _ = search(w.query())
    assert "call_value0" in defined(prog)


def test_keccak_interval_is_constructed():
    """A symbolic mapping key: ``lower <= f(x) < upper``, ``f(x) % 64 = 0``
    (keccak_function_manager.py's interval condition, ULE written as
    ``ult or =``) is met by construction, not by a 2^-123 guess."""
    w = W.World()
    t = w.tx()
    bal = t.sload(t.mapping(t.sender(), 0))
    t.require(S_uge(bal, t.arg(1)))
    prog, hits = search(w.query())
    names = defined(prog)
    assert any(n.startswith("keccak256_512#v0#") for n in names)
    assert hits > 0


def S_uge(a, b):
    from mythril_amd import smt as S
    return S.UGE(a, b)


def test_or_branches_cover_both_disjuncts():
    """``x = 7 or (y = 9 and x = 3)``: a selector commits each candidate to
    one disjunct; both are reached."""
    x, y = N.bv_var("x", 256), N.bv_var("y", 256)
    q = [N.bool_op("or", N.eq(x, N.bv_num(7, 256)),
                   N.bool_op("and", N.eq(y, N.bv_num(9, 256)), N.eq(x, N.bv_num(3, 256))))]
    prog, hits = search(q, n=64)
    assert "x" in defined(prog)
    assert hits == 64                      # every branch is a model
    seen = set()
    table = [sum(int(prog.consts[i, j]) << (32 * j) for j in range(8))
             for i in range(prog.consts.shape[0])]
    for idx in range(64):
        lv = [gen_ref.gen_leaf(11, 0, li, idx, l.width,
                               table[prog.pool_ranges[li][0]:sum(prog.pool_ranges[li])],
                               pct=(20, 40, 60)) for li, l in enumerate(prog.leaves)]
        _, probes = ir_sim.run(prog, lv)
        seen.add(unpack(prog, _pack1(lv), _pack1(probes)).vars["x"])
    assert seen == {3, 7}


def test_small_range_and_alignment():
    """``16 <= x < 4096 and x % 64 = 0`` — x = base + (aux << 6)."""
    x = N.bv_var("x", 256)
    q = [N.bv_cmp("bvuge", x, N.bv_num(16, 256)), N.bv_cmp("bvult", x, N.bv_num(4096, 256)),
         N.eq(N.bv_op("bvurem", x, N.bv_num(64, 256)), N.bv_num(0, 256))]
    prog, hits = search(q, n=64)
    assert "x" in defined(prog) and hits == 64


def test_definitions_never_make_unsat_sat():
    """``x = 5 and x = 6``: x is defined by the first equality, the second
    is still evaluated (no candidate passes)."""
    x = N.bv_var("x", 256)
    q = [N.eq(x, N.bv_num(5, 256)), N.eq(x, N.bv_num(6, 256))]
    prog, hits = search(q, n=32)
    assert hits == 0


@pytest.mark.parametrize("name", ["c1", "c3", "c4"])
def test_workload_witnesses_sound(name):
    """Independent groups of the stand-in shapes, as get_model splits them:
    every constructed candidate is judged exactly like the oracle judges its
    model; C1 / C4 groups are hit."""
    from mythril_amd.model import dependence_buckets
    hits = 0
    for q in W.queries(name, 12)[::4]:
        for g in dependence_buckets(q):
            try:
                _, h = search(g, n=24)
            except Exception as e:        # a group over the spill budget: plain search
                assert "spill budget" in str(e)
                continue
            hits += h
    if name != "c3":
        assert hits > 0


def _bec_batch_query(receivers):
    from mythril_amd.workloads import World, bv, ACTORS, _TOTAL, _BAL, _OWNER_PAUSED, _bec_batch
    w = World(concrete_storage=True)
    c = w.tx(creation=True)
    supply = bv(7000000000 * 10 ** 18)
    c.sstore(bv(_TOTAL), supply)
    c.sstore(c.mapping(bv(ACTORS[0]), _BAL), supply)
    c.sstore(bv(_OWNER_PAUSED), bv(ACTORS[0]))
    t = w.tx()
    checks = []
    _bec_batch(t, checks, receivers)
    return w.query([checks[0]])                # Not(BVMulNoOverflow(cnt, value))


def test_abi_offsets_are_preset():
    """batchTransfer(address[],uint256) reads _receivers at calldata[off + 4
    + i] with off the word at byte 4 (abi.py): off is pinned right after the
    head (0x40), calldatasize to the end of the last read, and every read
    becomes a constant-key read."""
    from mythril_amd import abi
    from mythril_amd.smt.node import topo_order
    q = _bec_batch_query(2)
    plan = abi.plan(q)
    assert plan is not None
    cells = plan.arrays["1_calldata"]
    assert [cells[4 + i] for i in range(32)] == list((0x40).to_bytes(32, "big"))
    assert plan.vars["1_calldatasize"] == 4 + 0x40 + 32 * 3        # length + two receivers
    q2 = plan.apply(q)
    sym = [n for n in topo_order(q2) if n.op == "select" and n.args[0].op == "array" and
           n.args[0].params[0] == "1_calldata" and n.args[1].op != "bvnum"]
    assert sym == []


def test_bec_batch_overflow_is_found():
    """The BECToken batchTransfer overflow (cnt = 2, value = 2^255, amount
    wraps to 0): the search program pins the ABI offsets, commits to the
    wrapping value and the joint bounds 2 <= cnt <= 2, and its witnesses
    are models of the original query (presets merged) in the oracle."""
    from mythril_amd.model import _compile_search, dependence_buckets
    q = _bec_batch_query(2)
    g = max(dependence_buckets(q), key=len)
    prog = _compile_search(g)
    assert prog.presets is not None and prog.solved
    table = [sum(int(prog.consts[i, j]) << (32 * j) for j in range(8))
             for i in range(prog.consts.shape[0])]
    hits = 0
    for idx in range(256):
        lv = [gen_ref.gen_leaf(11, 0, li, idx, l.width,
                               table[prog.pool_ranges[li][0]:sum(prog.pool_ranges[li])],
                               pct=(20, 40, 60)) for li, l in enumerate(prog.leaves)]
        root, probes = ir_sim.run(prog, lv)
        a = unpack(prog, _pack1(lv), _pack1(probes))
        assert root == R.eval_constraints(g, R.Assignment(a.vars, a.arrays, a.funcs)), idx
        hits += root
    assert hits > 0


@pytest.mark.parametrize("start", [0, 40, 80])
def test_solve_mode_sound_on_random_dags(start):
    """Fuzz: the C2 generator's random DAGs (every operator, arrays, 64-512
    nodes) compiled in search mode — folding, interval reasoning and every
    definition rule applied to shapes no workload builder produces.  On
    every candidate the program's root bit equals the oracle's verdict on
    the unpacked model of the ORIGINAL constraints."""
    from mythril_amd.corpus import make_dag
    from mythril_amd.ir import Unsupported
    checked = 0
    for d in range(start, start + 40):
        roots, _ = make_dag(d)
        try:
            prog = compile_constraints(roots, const_keys=True, leaf_pools=True, solve=True)
        except Unsupported:
            continue
        table = [sum(int(prog.consts[i, j]) << (32 * j) for j in range(8))
                 for i in range(prog.consts.shape[0])]
        for idx in range(6):
            lv = [gen_ref.gen_leaf(5, d, li, idx, l.width,
                                   table[prog.pool_ranges[li][0]:sum(prog.pool_ranges[li])],
                                   pct=(20, 40, 60)) for li, l in enumerate(prog.leaves)]
            root, probes = ir_sim.run(prog, lv)
            a = unpack(prog, _pack1(lv), _pack1(probes))
            assert root == R.eval_constraints(roots, R.Assignment(a.vars, a.arrays, a.funcs)), \
                (d, idx)
        checked += 1
    assert checked >= 30
