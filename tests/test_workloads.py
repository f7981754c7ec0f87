"""CPU checks of the C1 / C3 / C4 stand-in query builders
(mythril_amd/workloads.py): host Keccak against the oracle, planted models
that satisfy the paths the builders claim are feasible (pinning the lowering
against the reference's semantics through the oracle), and the compiled IR
(both table modes) against the oracle on every workload shape."""

import random

import numpy as np
import pytest

import ir_sim
from mythril_amd import workloads as W
from mythril_amd.assign import leaf_values, unpack
from mythril_amd.ir import compile_constraints
from oracle import gen_ref
from oracle import smtlib_ref as R
from oracle.keccak_ref import keccak256 as ref_keccak
from test_oracle_golden import load

ATTACKER, SOMEGUY, CREATOR = W.ACTORS[1], W.ACTORS[2], W.ACTORS[0]


def test_host_keccak_matches_oracle():
    for k in load("keccak_kat.json"):
        assert W.keccak256(bytes.fromhex(k["msg_hex"])).hex() == k["digest"][2:]
    rng = random.Random(4)
    for n in list(range(0, 70)) + [135, 136, 137, 300]:
        m = bytes(rng.randrange(256) for _ in range(n))
        assert W.keccak256(m) == ref_keccak(m)
    assert W.selector("transfer(address,uint256)") == 0xA9059CBB


def _calldata(sel, words):
    data = sel.to_bytes(4, "big") + b"".join(w.to_bytes(32, "big") for w in words)
    return [(i, b) for i, b in enumerate(data) if b], len(data)


def test_c1_kill_zero_path_is_satisfied_by_planted_model():
    w = W.World()
    t = w.tx()
    t.dispatch(W.SUICIDE_FUNCS, 0)
    t.jumpi(t.arg_address(0) == W.bv(0), taken=True)
    q = w.query()
    ents, size = _calldata(W.SUICIDE_FUNCS[0], [0])
    asg = R.Assignment(vars={"sender_0": ATTACKER, "call_value0": 0, "0_calldatasize": size},
                       arrays={"0_calldata": (ents, 0), "balance": ([], 0)})
    assert R.eval_constraints(q, asg) == 1
    bad = R.Assignment(vars=dict(asg.vars),
                       arrays={"0_calldata": (ents + [(35, 1)], 0), "balance": ([], 0)})
    assert R.eval_constraints(q, bad) == 0
    # short calldata: the selector bytes past the size read as 0
    short = R.Assignment(vars=dict(asg.vars, **{"0_calldatasize": 3}), arrays=asg.arrays)
    assert R.eval_constraints(q, short) == 0
    # a caller outside the three actors violates the setup constraint
    stranger = R.Assignment(vars=dict(asg.vars, sender_0=5), arrays=asg.arrays)
    assert R.eval_constraints(q, stranger) == 0


def test_c4_token_underflow_is_satisfied_by_planted_model():
    """token.sol transfer from an account holding nothing: the SUB underflow
    check (integer.py:157) is satisfiable once the keccak UF pair maps the
    sender's and receiver's mapping slots into the 512-bit interval."""
    w = W.World()
    c = w.tx(creation=True)
    supply = c.arg(0)
    c.sstore(W.bv(1), supply)
    c.sstore(c.mapping(W.bv(CREATOR), 0), supply)
    t = w.tx()
    checks = []
    W._token_transfer(t, checks)
    q = w.query([checks[0]])
    lo = w.kfm.interval_hook_for_size[512] * W.PART
    h_a = (lo + 63) // 64 * 64 + 64
    h_t = h_a + 64
    k_c, k_a, k_t = CREATOR << 256, ATTACKER << 256, SOMEGUY << 256
    h_c = int.from_bytes(W.keccak256(k_c.to_bytes(64, "big")), "big")
    ents, size = _calldata(W.TOKEN_FUNCS[W.TOKEN_FUNCS.index(W.selector("transfer(address,uint256)"))],
                           [SOMEGUY, 1])
    vars_ = {"sender_1": ATTACKER, "call_value1": 0, "1_calldatasize": size, "call_value0": 0,
             "0_calldatasize": 36}
    arrays = {"1_calldata": (ents, 0), "0_calldata": ([(35, 7)], 0), "balance": ([], 0)}
    funcs = {"keccak256_512": ([(k_c, h_c), (k_a, h_a), (k_t, h_t)], 0),
             "keccak256_512-1": ([(h_c, k_c), (h_a, k_a), (h_t, k_t)], 0)}
    asg = R.Assignment(vars=vars_, arrays=arrays, funcs=funcs)
    assert R.eval_constraints(q, asg) == 1
    # the underflow check itself is what the model satisfies: value 0 fails it
    ents0, _ = _calldata(W.TOKEN_FUNCS[W.TOKEN_FUNCS.index(W.selector("transfer(address,uint256)"))],
                         [SOMEGUY, 0])
    zero = R.Assignment(vars=vars_, arrays=dict(arrays, **{"1_calldata": (ents0, 0)}), funcs=funcs)
    assert R.eval_constraints(q, zero) == 0
    # a slot hash outside the 512-bit interval violates the keccak condition
    off = R.Assignment(vars=vars_, arrays=arrays,
                       funcs={"keccak256_512": ([(k_c, h_c), (k_a, h_a + 1), (k_t, h_t)], 0),
                              "keccak256_512-1": ([(h_c, k_c), (h_a + 1, k_a), (h_t, k_t)], 0)})
    assert R.eval_constraints(q, off) == 0


@pytest.mark.parametrize("name", ["c1", "c3", "c4", "c5"])
def test_workload_shapes(name):
    qs = W.queries(name, 48)
    assert len(qs) == 48
    ops = set()
    from mythril_amd.smt.node import topo_order
    for q in qs:
        for n in topo_order(q):
            ops.add(n.op)
    assert {"select", "ite", "concat", "bvslt", "bvult", "="} <= ops
    if name == "c3":
        assert {"bvumul_noovfl", "apply", "store", "K"} <= ops
    if name == "c4":
        assert {"apply", "store", "bvurem"} <= ops
    if name == "c5":
        assert {"apply", "store", "bvurem", "bvudiv", "bvumul_noovfl", "extract"} <= ops
    # deterministic
    assert [len(q) for q in W.queries(name, 48)] == [len(q) for q in qs]


def _to_oracle(prog, lv):
    arr = np.zeros((len(prog.leaves), 8), dtype=np.uint32)
    for i, v in enumerate(lv):
        for j in range(8):
            arr[i, j] = (v >> (32 * j)) & 0xFFFFFFFF
    a = unpack(prog, arr)
    return R.Assignment(a.vars, a.arrays, a.funcs)


@pytest.mark.parametrize("name,const_keys", [("c1", False), ("c1", True), ("c3", False),
                                             ("c3", True), ("c4", False), ("c4", True),
                                             ("c5", False), ("c5", True)])
def test_workload_programs_through_ir(name, const_keys):
    """Compiled IR (leaf-keyed or constant-keyed tables) executed by the
    reference executor equals direct oracle evaluation of the source DAG
    under generator candidates, pools included."""
    qs = W.queries(name, 40)[::5]
    for qi, q in enumerate(qs):
        prog = compile_constraints(q, const_keys=const_keys, leaf_pools=const_keys)
        table = [sum(int(prog.consts[i, j]) << (32 * j) for j in range(8))
                 for i in range(prog.consts.shape[0])]
        for idx in range(6):
            lv = []
            for li, l in enumerate(prog.leaves):
                off, n = prog.pool_ranges[li] if prog.pool_ranges else (0, len(prog.const_values))
                lv.append(gen_ref.gen_leaf(0xABC, qi, li, idx, l.width, table[off:off + n],
                                           pct=(20, 40, 60)))
            asg = _to_oracle(prog, lv)
            root, _ = ir_sim.run(prog, lv)
            assert root == R.eval_constraints(q, asg), (name, qi, idx)
            # the model packs back to leaves that evaluate the same (a
            # leaf-keyed entry at a constant key is shadowed, so it may move)
            back = leaf_values(prog, unpack(prog, _pack1(lv)))
            assert ir_sim.run(prog, back)[0] == root


def _pack1(lv):
    arr = np.zeros((len(lv), 8), dtype=np.uint32)
    for i, v in enumerate(lv):
        for j in range(8):
            arr[i, j] = (v >> (32 * j)) & 0xFFFFFFFF
    return arr


def test_const_keys_fold_constant_reads_to_leaves():
    from mythril_amd.smt import node as N
    cd = N.array_var("cd", 256, 8)
    x = N.bv_var("x", 256)
    q = [N.eq(N.select(cd, N.bv_num(3, 256)), N.bv_num(0x2A, 8)),
         N.eq(N.select(cd, x), N.bv_num(7, 8))]
    prog = compile_constraints(q, const_keys=True)
    assert prog.table_ckeys == {"cd": [3]}
    kinds = sorted(l.kind for l in prog.leaves)
    assert kinds.count("cval") == 1
    # model: cd[3] = 0x2A, x = 3 reads the same entry -> second constraint false
    lv_ok = {"cd#c0#0": 0x2A, "x": 9, "cd#k0#0": 9, "cd#v0#0": 7}
    lv = [lv_ok.get(l.name, 0) for l in prog.leaves]
    root, _ = ir_sim.run(prog, lv)
    assert root == 1 and R.eval_constraints(q, _to_oracle(prog, lv)) == 1
    lv_bad = dict(lv_ok, x=3)
    lv = [lv_bad.get(l.name, 0) for l in prog.leaves]
    root, _ = ir_sim.run(prog, lv)
    assert root == 0 and R.eval_constraints(q, _to_oracle(prog, lv)) == 0


def test_const_keys_skip_tables_read_at_many_symbolic_offsets():
    from mythril_amd.ir import scan_const_keys
    from mythril_amd.smt import node as N
    cd = N.array_var("cd", 256, 8)
    reads = [N.select(cd, N.bv_num(i, 256)) for i in range(40)]
    reads += [N.select(cd, N.bv_op("bvadd", N.bv_var("o", 256), N.bv_num(i, 256)))
              for i in range(60)]
    q = [N.eq(N.concat(*reads), N.bv_num(0, 800))]
    assert scan_const_keys(q) == {}
    assert scan_const_keys(q, max_links=10 ** 6)["cd"] == list(range(40))


@pytest.mark.parametrize("name", ["c1", "c3", "c4", "c5"])
def test_solve_mode_constructs_consistent_models(name):
    """Search-mode programs (argument-keyed tables + equality substitution)
    compute part of the model; under the model unpacked from leaves AND the
    computed probe values, the oracle's verdict on the ORIGINAL query equals
    the program's root bit on every candidate."""
    from mythril_amd.ir import Unsupported
    solved = 0
    for qi, q in enumerate(W.queries(name, 24)[::3]):
        try:
            prog = compile_constraints(q, const_keys=True, leaf_pools=True, solve=True)
        except Unsupported as e:       # over the spill budget: get_model searches plain
            assert "spill budget" in str(e)
            continue
        solved += prog.solved
        table = [sum(int(prog.consts[i, j]) << (32 * j) for j in range(8))
                 for i in range(prog.consts.shape[0])]
        for idx in range(8):
            lv = []
            for li, l in enumerate(prog.leaves):
                off, n = prog.pool_ranges[li]
                lv.append(gen_ref.gen_leaf(7, qi, li, idx, l.width, table[off:off + n],
                                           pct=(20, 40, 60)))
            root, probes = ir_sim.run(prog, lv)
            a = unpack(prog, _pack1(lv), _pack1(probes))
            assert root == R.eval_constraints(q, R.Assignment(a.vars, a.arrays, a.funcs)), (qi, idx)
    assert solved > 0


def test_solve_mode_defines_keccak_inverse_and_size():
    """keccak256_N-1(keccak256_N(x)) = x and calldatasize = 64 become
    definitions, not guesses (keccak_function_manager.py:145-149,
    instructions.py:1020-1025)."""
    from mythril_amd.smt import node as N
    w = W.World()
    t = w.tx()
    w.constraints.append(t.calldata.size == W.bv(64))
    t.mapping(t.sender(), 0)
    q = w.query()
    prog = compile_constraints(q, const_keys=True, leaf_pools=True, solve=True)
    names = {prog.leaves[li].name for li in prog.derived}
    assert "0_calldatasize" in names
    assert any(n.startswith("keccak256_512-1#v0#") for n in names)
    assert "keccak256_512" in prog.entry_keys and "keccak256_512-1" in prog.entry_keys
    # a model built from any candidate satisfies those two conjuncts by construction
    lv = [0] * len(prog.leaves)
    root, probes = ir_sim.run(prog, lv)
    a = unpack(prog, _pack1(lv), _pack1(probes))
    asg = R.Assignment(a.vars, a.arrays, a.funcs)
    assert R.eval_constraints([q[-2]], asg) == 1        # calldatasize == 64
    inv_eq = [c for c in q if c.op == "and"][-1].args[0]  # inv(f(x)) == x of the keccak condition
    assert R.eval_constraints([inv_eq], asg) == 1


def test_reference_keccak_val8_sym256_case_is_satisfiable():
    """tests/laser/keccak_tests.py:23-27 (reference) expects unsat for
    keccak(100_8) == keccak(N1_256), but under the encoding the reference's
    keccak_function_manager builds (its concrete-hash branch compares the
    8-bit key with N1 zero-padded, keccak_function_manager.py:146-148 and
    bitvec.py:16-22) the query has a model; the oracle checks it here."""
    from mythril_amd.smt import And, symbol_factory
    km = W.KeccakFunctionManager(ref_keccak)
    o1, c1 = km.create_keccak(symbol_factory.BitVecVal(100, 8))
    o2, c2 = km.create_keccak(symbol_factory.BitVecSym("N1", 256))
    q = [And(c1, c2).raw, (o1 == o2).raw]
    h = int.from_bytes(ref_keccak(bytes([100])), "big")
    asg = R.Assignment(vars={"N1": 100},
                       funcs={"keccak256_256": ([(100, h)], 0), "keccak256_256-1": ([(h, 100)], 0),
                              "keccak256_8": ([(100, h)], 0), "keccak256_8-1": ([(h, 100)], 0)})
    assert R.eval_constraints(q, asg) == 1


def test_c5_interleaves_all_thirteen_contracts():
    """C5 = every solidity_examples contract: twelve streams (token and
    WalletLibrary share C4's), the first 12 queries are one from each stream
    in C5_CONTRACTS order, and every one of the nine C5-only contracts builds
    queries that compile."""
    assert len(W.C5_CONTRACTS) == 12 and len(W.C5_EXTRA) == 9
    per = 2
    firsts = [W.c1_queries(per, 0xC5 ^ 0xC1)[0], W.c3_queries(per, 0xC5 ^ 0xC3)[0],
              W.c4_queries(per, 0xC5 ^ 0xC4)[0]]
    firsts += [W.contract_queries(n, per, 0xC5 ^ (0x100 + k))[0]
               for k, n in enumerate(W.C5_EXTRA)]
    got = W.c5_queries(12 * per)[:12]
    assert [[c.id for c in q] for q in got] == [[c.id for c in q] for q in firsts]
    for name in W.C5_EXTRA:
        for q in W.contract_queries(name, 6, 3):
            compile_constraints(q)
            compile_constraints(q, const_keys=True, leaf_pools=True)
