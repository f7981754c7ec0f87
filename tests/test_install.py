"""install() against a stand-in ``mythril`` package (the real one needs z3 and
is not importable here): every binding INTEGRATION.md lists is rebound, the
singletons are adopted, the statistics class is patched, and queries keep
flowing through the rebound names.  The stand-in modules carry only the
names install() touches."""

import sys
import types

import pytest

import mythril_amd.model as M


class _Args:
    solver_timeout = 10000
    sparse_pruning = True


class _TimeHandler:
    def time_remaining(self):
        return 60_000


class _StatsStub:
    def __init__(self):
        self.enabled = True
        self.query_count = 0
        self.solver_time = 0.0

    def __repr__(self):
        return "Query count: {} \nSolver time: {}".format(self.query_count, self.solver_time)


def _stub(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    return m


@pytest.fixture
def fake_mythril(monkeypatch):
    args, th = _Args(), _TimeHandler()
    mods = {
        "mythril": _stub("mythril"),
        "mythril.support": _stub("mythril.support"),
        "mythril.support.support_args": _stub("mythril.support.support_args", args=args),
        "mythril.support.model": _stub("mythril.support.model", get_model=lambda *a, **k: None),
        "mythril.laser": _stub("mythril.laser"),
        "mythril.laser.ethereum": _stub("mythril.laser.ethereum"),
        "mythril.laser.ethereum.time_handler": _stub("mythril.laser.ethereum.time_handler",
                                                     time_handler=th),
        "mythril.laser.ethereum.state": _stub("mythril.laser.ethereum.state"),
        "mythril.laser.ethereum.state.constraints": _stub(
            "mythril.laser.ethereum.state.constraints", get_model=lambda *a, **k: None),
        "mythril.laser.ethereum.keccak_function_manager": _stub(
            "mythril.laser.ethereum.keccak_function_manager", keccak_function_manager=object()),
        "mythril.laser.smt": _stub("mythril.laser.smt", Optimize=object, Model=object,
                                   symbol_factory=object()),
        "mythril.laser.smt.solver": _stub("mythril.laser.smt.solver"),
        "mythril.laser.smt.solver.solver_statistics": _stub(
            "mythril.laser.smt.solver.solver_statistics", SolverStatistics=_StatsStub),
        "mythril.analysis": _stub("mythril.analysis"),
        "mythril.analysis.solver": _stub("mythril.analysis.solver",
                                         get_model=lambda *a, **k: None,
                                         _replace_with_actual_sha=lambda *a, **k: None),
    }
    for name, mod in mods.items():
        monkeypatch.setitem(sys.modules, name, mod)
    # install() rebinds these module globals: restore them afterwards
    for g in ("args", "time_handler", "_stock_optimize", "_stock_model"):
        monkeypatch.setattr(M, g, getattr(M, g))
    monkeypatch.setattr(M, "GPU_ENABLED", M.GPU_ENABLED)
    monkeypatch.setattr(M, "DEVICES", list(M.DEVICES))
    return mods, args, th


def test_install_rebinds_every_get_model_name(fake_mythril):
    mods, args, th = fake_mythril
    M.install()
    for name in ("mythril.support.model", "mythril.analysis.solver",
                 "mythril.laser.ethereum.state.constraints"):
        assert mods[name].get_model is M.get_model, name
    assert M.args is args and M.time_handler is th
    assert M._stock_optimize is mods["mythril.laser.smt"].Optimize
    assert M._stock_model is mods["mythril.laser.smt"].Model
    # the concrete-hash walk of reported transactions goes through the GPU batch
    assert mods["mythril.analysis.solver"]._replace_with_actual_sha.__module__ == M.__name__


def test_install_patches_solver_statistics(fake_mythril):
    mods, _, _ = fake_mythril
    M.install()
    stats = mods["mythril.laser.smt.solver.solver_statistics"].SolverStatistics()
    text = repr(stats)
    assert text.startswith("Query count: 0 \nSolver time: 0.0")        # the reference's lines
    assert "GPU" in text                                                # then the pre-filter's


def test_install_reads_the_environment(fake_mythril, monkeypatch):
    monkeypatch.setenv("MYTHRIL_GPU", "0")
    monkeypatch.setenv("MYTHRIL_GPU_DEVICES", "0,1")
    M.install()
    assert M.GPU_ENABLED is False and M.DEVICES == [0, 1]


def test_installed_get_model_answers_python_bools(fake_mythril):
    """Through the rebound name, Python-bool handling is the reference's
    (support/model.py:32-37): a False constraint is unsat without any
    solver, True ones are dropped."""
    mods, _, _ = fake_mythril
    M.install()
    gm = mods["mythril.laser.ethereum.state.constraints"].get_model
    gm.cache_clear()
    with pytest.raises(M.UnsatError):
        gm((False,))
