"""Host compiler checks on the CPU: compiled IR executed by the reference
executor (tests/ir_sim.py) must equal direct oracle evaluation of the source
DAG, for every probe and the root, on every case."""

import random

import numpy as np
import pytest

import dag_cases
import ir_sim
from evm_mini import lower_program
from mythril_amd import irdefs as I
from mythril_amd.assign import Assignment as PAssignment, leaf_values, pack, unpack
from mythril_amd.corpus import make_dag
from mythril_amd.ir import Unsupported, compile_constraints
from mythril_amd.smt import node as N
from oracle import gen_ref
from oracle import smtlib_ref as R
from test_oracle_golden import load, oracle_eval

CASES = dag_cases.named_cases()


def to_product(asg: R.Assignment) -> PAssignment:
    return PAssignment(asg.vars, asg.arrays, asg.funcs)


def check_program(prog, constraints, probes, assignments):
    for asg in assignments:
        lv = leaf_values(prog, to_product(asg))
        root, got = ir_sim.run(prog, lv)
        want = R.evaluate(list(probes), asg)
        # probes of width > 256 come out as consecutive 256-bit chunks
        flat = []
        for p, v in zip(probes, want):
            for k in range((p.width + 255) // 256):
                flat.append((v >> (256 * k)) & ((1 << min(256, p.width - 256 * k)) - 1))
        assert got == flat, (asg, [(i, g, w) for i, (g, w) in enumerate(zip(got, flat)) if g != w][:3])
        assert root == R.eval_constraints(constraints, asg)


@pytest.mark.parametrize("name", sorted(CASES))
def test_case_through_ir(name):
    constraints, probes, gen, tables = CASES[name]
    prog = compile_constraints(constraints, probes, table_sizes=tables)
    rng = random.Random(hash(name) & 0xFFFF)
    check_program(prog, constraints, probes, [gen(rng) for _ in range(60)])


@pytest.mark.parametrize("t", load("vmtests.json")[::3], ids=lambda t: t["name"])
def test_vmtest_through_ir(t):
    vars_, stores, divergent = lower_program(t["code"], oracle_eval)
    probes = [v.raw for _, v in stores] + [k.raw for k, _ in stores]
    prog = compile_constraints([], probes)
    asg = R.Assignment(vars=vars_)
    lv = leaf_values(prog, to_product(asg))
    _, got = ir_sim.run(prog, lv)
    n = len(stores)
    storage = {}
    for k, v in zip(got[n:], got[:n]):
        storage[k] = v
    storage = {k: v for k, v in storage.items() if v}
    if not divergent:
        assert storage == {int(k, 16): int(v, 16) for k, v in t["storage"].items()}


@pytest.mark.parametrize("dag_id", range(0, 40, 3))
def test_corpus_dag_through_ir(dag_id):
    roots, _ = make_dag(dag_id)
    prog = compile_constraints(roots)
    assert prog.stats["lnodes"] > 0
    pool = prog.const_values
    for idx in range(12):
        lv = [gen_ref.gen_leaf(0x1234, dag_id, li, idx, l.width, pool)
              for li, l in enumerate(prog.leaves)]
        asg = to_oracle(prog, lv)
        root, _ = ir_sim.run(prog, lv)
        assert root == R.eval_constraints(roots, asg)


def to_oracle(prog, lv):
    arr = np.zeros((len(prog.leaves), 8), dtype=np.uint32)
    for i, v in enumerate(lv):
        for j in range(8):
            arr[i, j] = (v >> (32 * j)) & 0xFFFFFFFF
    a = unpack(prog, arr)
    return R.Assignment(a.vars, a.arrays, a.funcs)


def test_code_invariants():
    roots, _ = make_dag(5)
    prog = compile_constraints(roots)
    code = prog.code
    ops = code[:, 0] & 0xFF
    assert (ops < I.NUM_OPS).all()
    for k in range(4):
        assert (((code[:, 1] >> (8 * k)) & 0xFF) < I.NREG).all()
    assert prog.n_lds <= I.MAX_LDS + I.MAX_PSLOTS
    fused = (code[:, 0] & I.ROOT_FLAG) != 0
    assert (ops == I.ROOT).sum() + fused.sum() == len(roots)
    assert fused.sum() > 0


def test_pack_unpack_roundtrip():
    constraints, probes, gen, tables = CASES["keccak_uf"]
    prog = compile_constraints(constraints, probes, table_sizes=tables)
    rng = random.Random(3)
    asgs = [to_product(gen(rng)) for _ in range(5)]
    soa = pack(prog, asgs)
    assert soa.shape == (len(prog.leaves), 8, 5)
    for a in range(5):
        back = unpack(prog, soa[:, :, a])
        assert leaf_values(prog, back) == leaf_values(prog, asgs[a])


def test_unsupported_array_equality():
    A, B = N.array_var("A", 256, 256), N.array_var("B", 256, 256)
    with pytest.raises(Unsupported):
        compile_constraints([N.eq(A, B)])


def test_wide_arithmetic_is_unsupported():
    x = N.bv_var("w512", 512)
    with pytest.raises(Unsupported):
        compile_constraints([N.eq(N.bv_op("bvadd", x, x), x)])


def test_deep_concat_chain_compiles():
    # a 32-byte calldata-style word: 31 CONCATs, and a deep chain of adds
    bytes_ = [N.bv_var("b%d" % i, 8) for i in range(32)]
    w = N.concat(*bytes_)
    acc = w
    for i in range(3000):
        acc = N.bv_op("bvadd", acc, N.bv_num(i, 256))
    prog = compile_constraints([N.bv_cmp("bvult", acc, w)])
    assert prog.n_ins > 3000


# ---- constraint-guided candidate pools (search mode) -------------------------

def _table_values(prog):
    return [sum(int(prog.consts[i, j]) << (32 * j) for j in range(8))
            for i in range(prog.consts.shape[0])]


def test_leaf_pools_follow_comparisons():
    """A leaf's pool holds the constants it is compared with (and their byte
    slices for narrow leaves), not the query's other constants."""
    bs = [N.bv_var("b%d" % i, 8) for i in range(4)]
    x, y = N.bv_var("x", 256), N.bv_var("y", 256)
    cons = [N.eq(N.concat(*bs), N.bv_num(0xA9059CBB, 32)),
            N.eq(x, N.bv_num(0xDEADBEEF, 256)),
            N.bv_cmp("bvult", y, N.bv_num(1000, 256))]
    plain = compile_constraints(cons)
    prog = compile_constraints(cons, leaf_pools=True)
    # the CONST prefix is that of the plain compile; pools only follow it
    assert prog.const_values == plain.const_values
    assert prog.n_ins == plain.n_ins
    assert _table_values(prog)[:len(prog.const_values)] == prog.const_values
    table = _table_values(prog)
    idx = prog.leaf_index()
    pools = {}
    for name, li in idx.items():
        off, n = prog.pool_ranges[li]
        assert 0 < n and off + n <= len(table)
        pools[name] = set(table[off:off + n])
    for i in range(4):
        assert {0xA9, 0x05, 0x9C, 0xBB} <= pools["b%d" % i]
        assert 0xDEADBEEF not in pools["b%d" % i]
    assert 0xDEADBEEF in pools["x"] and 1000 not in pools["x"]
    assert 1000 in pools["y"] and 1024 in pools["y"] and 0xDEADBEEF not in pools["y"]


def test_leaf_without_constant_comparison_uses_whole_table():
    x, y = N.bv_var("x", 256), N.bv_var("y", 256)
    cons = [N.bv_cmp("bvult", x, y), N.eq(N.bv_op("bvadd", x, N.bv_num(5, 256)), N.bv_num(9, 256))]
    prog = compile_constraints(cons, leaf_pools=True)
    li = prog.leaf_index()
    assert prog.pool_ranges[li["y"]] == (0, len(prog.const_values))
    off, n = prog.pool_ranges[li["x"]]
    assert {5, 9} <= set(_table_values(prog)[off:off + n])


@pytest.mark.parametrize("dag_id", [1, 7, 20])
def test_corpus_dag_with_leaf_pools_through_ir(dag_id):
    """Per-leaf pools only add table entries: the program still evaluates
    exactly the DAG under generator values drawn from them."""
    roots, _ = make_dag(dag_id)
    prog = compile_constraints(roots, leaf_pools=True)
    table = _table_values(prog)
    for idx in range(12):
        lv = []
        for li, l in enumerate(prog.leaves):
            off, n = prog.pool_ranges[li]
            lv.append(gen_ref.gen_leaf(0x1234, dag_id, li, idx, l.width, table[off:off + n],
                                       pct=(20, 40, 60)))
        asg = to_oracle(prog, lv)
        root, _ = ir_sim.run(prog, lv)
        assert root == R.eval_constraints(roots, asg)


def test_auto_leaf_policy_picks_per_program():
    """leaf_remat="auto" (the eval-mode batch compile): "always" for a
    program with almost no heavy arithmetic (ir.AUTO_ALWAYS_HEAVY), else
    scratch2, unless the program's 256-bit scratch reloads exceed
    ir.AUTO_SCRATCH_SHARE of its instructions — then "scratch"."""
    import numpy as np
    import bench
    from mythril_amd import ir
    picked = []
    for w, d in (("c2", 3), ("c2", 5), ("c3", 0), ("c3", 4), ("c4", 8)):
        roots = bench.workload_roots(w, d)
        auto = ir.compile_constraints(roots, leaf_remat="auto")
        s2 = ir.compile_constraints(roots, leaf_remat="scratch2")
        if ir.heavy_share(s2) < ir.AUTO_ALWAYS_HEAVY:
            pol = "always"
        elif ir.scratch_reload_share(s2) > ir.AUTO_SCRATCH_SHARE:
            pol = "scratch"
        else:
            pol = "scratch2"
        want = ir.compile_constraints(roots, leaf_remat=pol)
        assert np.array_equal(auto.code, want.code) and np.array_equal(auto.consts, want.consts)
        picked.append((w, pol))
    assert all(p != "always" for w, p in picked if w == "c2")     # VALU-bound: spills stay
    assert all(p == "always" for w, p in picked if w != "c2")
