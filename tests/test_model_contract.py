"""The drop-in get_model keeps the reference contract
(mythril/support/model.py:15-49) — checked with a fake GPU search on the CPU."""

import pytest

import mythril_amd.model as M
from mythril_amd.assign import Assignment
from mythril_amd.smt import ULT, symbol_factory


@pytest.fixture(autouse=True)
def fresh(monkeypatch):
    M.get_model.cache_clear()
    calls = []

    def fake_search(nodes, budget_ms):
        calls.append(nodes)
        if any(getattr(n, "op", "") == "false" for n in nodes):
            return None
        return Assignment(vars={"x": 1}), None
    monkeypatch.setattr(M, "gpu_search", fake_search)
    monkeypatch.setattr(M.z3bridge, "available", lambda: False)
    M.args.solver_timeout = 10000
    M.time_handler.start_execution(3600)
    yield calls
    M.get_model.cache_clear()


def c_sat():
    x = symbol_factory.BitVecSym("x", 256)
    return ULT(x, symbol_factory.BitVecVal(5, 256))


def test_timeout_exhausted_raises_before_any_work(fresh):
    M.time_handler.start_execution(0)          # no time left
    with pytest.raises(M.UnsatError):
        M.get_model((c_sat(),))
    assert fresh == []


def test_enforce_execution_time_false_ignores_deadline(fresh):
    M.time_handler.start_execution(0)
    m = M.get_model((c_sat(),), enforce_execution_time=False)
    assert m.assignment.vars["x"] == 1


def test_python_false_is_unsat(fresh):
    with pytest.raises(M.UnsatError):
        M.get_model((c_sat(), False))
    assert fresh == []


def test_python_true_is_dropped(fresh):
    M.get_model((True, c_sat()))
    assert len(fresh) == 1 and len(fresh[0]) == 1


def test_gpu_hit_returns_model_and_is_cached(fresh):
    c = (c_sat(),)
    m1 = M.get_model(c)
    m2 = M.get_model(c)
    assert m1 is m2 and len(fresh) == 1
    assert m1["x"] == 1


def test_miss_without_z3_never_claims_unsat(fresh):
    with pytest.raises(M.SolverUnavailable):
        M.get_model((symbol_factory.Bool(False).__class__(symbol_factory.Bool(False).raw),))


def test_optimize_queries_never_use_the_gpu(fresh):
    x = symbol_factory.BitVecSym("x", 256)
    with pytest.raises(M.SolverUnavailable):
        M.get_model((c_sat(),), minimize=(x,))
    assert fresh == []


def test_unsupported_falls_back(monkeypatch, fresh):
    from mythril_amd.ir import Unsupported

    def boom(nodes, budget_ms):
        raise Unsupported("x")
    monkeypatch.setattr(M, "gpu_search", boom)
    with pytest.raises(M.SolverUnavailable):
        M.get_model((c_sat(),))
    assert M.stats.unsupported >= 1
