"""The z3 bridge (mythril_amd/z3bridge.py) against an in-repo stand-in of the
z3 API (tests/fake_z3.py; z3 itself is not installed here): every §8a
declaration name round-trips through to_node / to_z3 (z3's internal ``*_i``
divisions and ``if`` included), the walks are linear on hash-consed DAGs
with 2^30 tree paths, and verify() accepts exactly the witnesses under which
substitute + simplify gives True — arrays and UFs included — before it asks
a Solver for the model."""

import sys

import pytest

import fake_z3 as Z
from mythril_amd import z3bridge
from mythril_amd.assign import Assignment
from mythril_amd.smt import node as N


@pytest.fixture(autouse=True)
def z3_stand_in(monkeypatch):
    monkeypatch.setitem(sys.modules, "z3", Z)
    yield


def _x(name="x", w=256):
    return Z.BitVec(name, w)


BV2 = {"bvadd": lambda a, b: a + b, "bvsub": lambda a, b: a - b, "bvmul": lambda a, b: a * b,
       "bvudiv": Z.UDiv, "bvsdiv": lambda a, b: a / b, "bvurem": Z.URem, "bvsrem": Z.SRem,
       "bvsmod": lambda a, b: a % b, "bvand": lambda a, b: a & b, "bvor": lambda a, b: a | b,
       "bvxor": lambda a, b: a ^ b, "bvshl": lambda a, b: a << b, "bvlshr": Z.LShR,
       "bvashr": lambda a, b: a >> b}
CMP = {"bvult": Z.ULT, "bvule": Z.ULE, "bvugt": Z.UGT, "bvuge": Z.UGE,
       "bvslt": lambda a, b: a < b, "bvsle": lambda a, b: a <= b, "bvsgt": lambda a, b: a > b,
       "bvsge": lambda a, b: a >= b, "bvumul_noovfl": lambda a, b: Z.BVMulNoOverflow(a, b, False)}


def _cases():
    x, y = _x(), _x("y")
    p, q = Z.Bool("p"), Z.Bool("q")
    A = Z.Array("A", Z.BitVecSort(256), Z.BitVecSort(8))
    f = Z.Function("keccak256_512", Z.BitVecSort(512), Z.BitVecSort(256))
    out = {}
    for name, fn in BV2.items():
        out[name] = (fn(x, y), name)
    for name, fn in CMP.items():
        out[name] = (fn(x, y), name)
    for zi, ours in (("bvudiv_i", "bvudiv"), ("bvsdiv_i", "bvsdiv"), ("bvurem_i", "bvurem"),
                     ("bvsrem_i", "bvsrem"), ("bvsmod_i", "bvsmod")):
        out[zi] = (Z.interpreted(zi, x.sort(), x, y), ours)
    out.update({
        "bvneg": (-x, "bvneg"), "bvnot": (~x, "bvnot"),
        "=": (x == y, "="), "distinct": (Z.Distinct(x, y, _x("z")), "distinct"),
        "if": (Z.If(p, x, y), "ite"), "and": (Z.And(p, q), "and"), "or": (Z.Or(p, q), "or"),
        "not": (Z.Not(p), "not"), "xor": (Z.Xor(p, q), "xor"), "=>": (Z.Implies(p, q), "=>"),
        "concat": (Z.Concat(Z.Extract(7, 0, x), _x("b", 8)), "concat"),
        "extract": (Z.Extract(200, 9, x), "extract"),
        "zero_extend": (Z.ZeroExt(56, _x("w", 200)), "zero_extend"),
        "sign_extend": (Z.SignExt(56, _x("w", 200)), "sign_extend"),
        "select": (Z.Select(A, x), "select"),
        "store/const": (Z.Select(Z.Store(Z.K(Z.BitVecSort(256), Z.BitVecVal(0, 8)), x,
                                         Z.BitVecVal(3, 8)), y), "select"),
        "uf": (f(Z.Concat(x, y)), "apply"),
        "true": (Z.BoolVal(True), "true"), "false": (Z.BoolVal(False), "false"),
        "numeral": (Z.BitVecVal(12345, 77), "bvnum"),
    })
    return out


@pytest.mark.parametrize("decl", sorted(_cases()))
def test_every_decl_round_trips(decl):
    e, ours = _cases()[decl]
    n = z3bridge.to_node(e, {})
    assert n.op == ours
    back = z3bridge.to_z3(n, {})
    assert z3bridge.to_node(back, {}) is n          # structural identity (hash-consed DAG)
    if decl.endswith("_i"):                          # z3's internal division names normalise
        assert back.decl().name() == ours


def test_params_are_kept():
    n = z3bridge.to_node(Z.Extract(200, 9, _x()), {})
    assert n.params == (200, 9) and n.width == 192
    n = z3bridge.to_node(Z.ZeroExt(56, _x("w", 200)), {})
    assert n.width == 256


def test_unknown_decl_is_unsupported():
    from mythril_amd.ir import Unsupported
    with pytest.raises(Unsupported):
        z3bridge.to_node(Z.interpreted("bvredor", Z.BitVecSort(1), _x()), {})


def _tower(levels):
    x = _x("t")
    for _ in range(levels):
        x = x + x                                    # 2^levels tree paths, levels + 1 nodes
    return x


def test_walks_are_linear_on_shared_dags():
    c = Z.ULT(_tower(30), Z.BitVecVal(5, 256))
    Z.CALLS["children"] = 0
    z3bridge.to_node(c, {})
    assert Z.CALLS["children"] < 200
    Z.CALLS["children"] = 0
    consts, funcs = z3bridge._symbols([c, c])
    assert [k.decl().name() for k in consts] == ["t"] and funcs == {}
    assert Z.CALLS["children"] < 100


def test_verify_substitutes_and_simplifies_before_the_solver():
    x = _x()
    c = [Z.ULT(x, Z.BitVecVal(10, 256)), x * x == Z.BitVecVal(49, 256)]
    m = z3bridge.verify(c, Assignment(vars={"x": 7}), 1000)
    assert m is not None and m["x"].as_long() == 7
    assert z3bridge.verify(c, Assignment(vars={"x": 6}), 1000) is None


def test_verify_on_a_deep_shared_dag_is_fast():
    c = [_tower(30) == Z.BitVecVal(3 << 30, 256)]
    Z.CALLS["children"] = 0
    assert z3bridge.verify(c, Assignment(vars={"t": 3}), 1000) is not None
    assert Z.CALLS["children"] < 1000


def test_verify_interprets_arrays_and_ufs_from_the_witness():
    x = _x()
    A = Z.Array("A", Z.BitVecSort(256), Z.BitVecSort(256))
    f = Z.Function("keccak256_256", Z.BitVecSort(256), Z.BitVecSort(256))
    c = [Z.Select(Z.Store(A, Z.BitVecVal(1, 256), Z.BitVecVal(5, 256)), x) == Z.BitVecVal(7, 256),
         f(x) == Z.BitVecVal(64, 256), f(Z.BitVecVal(1, 256)) == Z.BitVecVal(0, 256)]
    good = Assignment(vars={"x": 2}, arrays={"A": ([(2, 7)], 0)},
                      funcs={"keccak256_256": ([(2, 64)], 0)})
    assert z3bridge.verify(c, good, 1000) is not None
    # first match wins, as on the device
    shadowed = Assignment(vars={"x": 2}, arrays={"A": ([(2, 7), (2, 9)], 0)},
                          funcs={"keccak256_256": ([(2, 64)], 0)})
    assert z3bridge.verify(c, shadowed, 1000) is not None
    wrong_array = Assignment(vars={"x": 2}, arrays={"A": ([(2, 8)], 0)},
                             funcs={"keccak256_256": ([(2, 64)], 0)})
    assert z3bridge.verify(c, wrong_array, 1000) is None
    wrong_uf_default = Assignment(vars={"x": 2}, arrays={"A": ([(2, 7)], 0)},
                                  funcs={"keccak256_256": ([(2, 64)], 5)})
    assert z3bridge.verify(c, wrong_uf_default, 1000) is None   # f(1) falls to else = 5


def test_symbols_absent_from_the_witness_default_to_zero():
    x, y = _x(), _x("unused")
    c = [Z.ULT(x, Z.BitVecVal(3, 256)), Z.ULE(y, Z.BitVecVal(0, 256))]
    assert z3bridge.verify(c, Assignment(vars={"x": 1}), 1000) is not None


def test_get_model_verifies_gpu_witness_with_z3(monkeypatch):
    import mythril_amd.model as M
    monkeypatch.setattr(M.z3bridge, "available", lambda: True)
    x = _x("gx")
    c = (Z.ULT(x, Z.BitVecVal(10, 256)), x + x == Z.BitVecVal(14, 256))
    answers = iter([Assignment(vars={"gx": 7}), Assignment(vars={"gx": 8})])
    monkeypatch.setattr(M, "gpu_search", lambda nodes, budget_ms: (next(answers), []))
    fallbacks = []

    def fake_z3(constraints, minimize, maximize, timeout):
        fallbacks.append(timeout)
        raise M.UnsatError
    monkeypatch.setattr(M, "_z3_check", fake_z3)
    M.get_model.cache_clear()
    M.time_handler.start_execution(3600)
    m = M.get_model(c)
    assert m.raw and m.raw[0]["gx"].as_long() == 7 and not fallbacks
    rejected = M.stats.rejected
    M.get_model.cache_clear()
    with pytest.raises(M.UnsatError):                # the wrong witness goes to z3
        M.get_model(c)
    assert M.stats.rejected == rejected + 1 and len(fallbacks) == 1
    M.get_model.cache_clear()
