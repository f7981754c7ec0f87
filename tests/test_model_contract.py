"""The drop-in get_model keeps the reference contract
(mythril/support/model.py:15-49) — checked with a fake GPU search on the CPU."""

import pytest

import mythril_amd.model as M
from mythril_amd.assign import Assignment
from mythril_amd.smt import ULT, symbol_factory

REAL_GPU_SEARCH = M.gpu_search          # the fixture below swaps in a fake


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


# ---- batched is_possible ---------------------------

class FakeEngine:
    """Stands in for the GPU: a set is 'found' unless its program has no
    leaves (a constant query such as Bool false)."""

    def __init__(self):
        self.batches = []

    def load(self, prog, leafgen, prog_seed=0):
        return prog

    def batch_search(self, loaded, seed, n_cand, first_index=0, want_probes=False):
        self.batches.append(len(loaded))
        import numpy as np
        out = []
        for prog in loaded:
            unsat = len(prog.leaves) == 0               # e.g. a constant-false query
            hit = (-1, None) if unsat else (7, np.zeros((len(prog.leaves), 8), np.uint32))
            # (no batched probes here: the model asks witness() per hit)
            out.append(hit + (None,) if want_probes else hit)
        return out

    def witness(self, prog, seed, index):
        # a solve-mode program computes part of its model (x < 5 makes x a
        # small range): the values one re-evaluated lane reports
        import numpy as np
        import ir_sim
        _, probes = ir_sim.run(prog, [0] * len(prog.leaves))
        pr = np.zeros((len(probes), 8), np.uint32)
        for k, v in enumerate(probes):
            pr[k] = [(v >> (32 * j)) & 0xFFFFFFFF for j in range(8)]
        return np.zeros((len(prog.leaves), 8), np.uint32), pr


@pytest.fixture
def batch_env(monkeypatch, fresh):
    eng = FakeEngine()
    monkeypatch.setattr(M, "get_engine", lambda dev=0, slot=0: eng)
    z3_calls = []

    def fake_z3(constraints, minimize, maximize, timeout):
        z3_calls.append(constraints)
        raise M.UnsatError                         # z3 says unsat for every miss
    monkeypatch.setattr(M, "_z3_check", fake_z3)
    return eng, z3_calls


def test_witness_probes_from_the_batched_search_need_no_per_hit_launch(batch_env, monkeypatch):
    """A solve-mode hit whose probe values came back with the batched search
    (mg_batch_search_probes) is unpacked from them: no per-hit witness()."""
    eng, _ = batch_env
    import numpy as np
    import ir_sim

    def batch_search(loaded, seed, n_cand, first_index=0, want_probes=False):
        assert want_probes
        out = []
        for prog in loaded:
            lv = np.zeros((len(prog.leaves), 8), np.uint32)
            _, probes = ir_sim.run(prog, [0] * len(prog.leaves))
            pr = np.zeros((max(1, len(probes)), 8), np.uint32)
            for k, v in enumerate(probes):
                pr[k] = [(v >> (32 * j)) & 0xFFFFFFFF for j in range(8)]
            out.append((7, lv, pr))
        return out

    def no_witness(*a, **k):
        raise AssertionError("per-hit witness launch")
    monkeypatch.setattr(eng, "batch_search", batch_search)
    monkeypatch.setattr(eng, "witness", no_witness)
    m = M.get_model((c_sat(),))
    assert m.assignment.vars["x"] < 5           # a derived value, from the probes


def test_batch_is_possible_matches_the_per_state_loop(batch_env, monkeypatch):
    eng, z3_calls = batch_env
    x = symbol_factory.BitVecSym("x", 256)
    unsat_like = symbol_factory.Bool(False).__class__(symbol_factory.Bool(False).raw)
    sets = [(c_sat(),), (c_sat(), False), (unsat_like,), (True, c_sat()), (ULT(x, x),)]
    got = M.batch_is_possible(sets)
    # one batched search, no per-set launches; the constant-false set folds
    # on the host (no launch: model.search_groups)
    assert eng.batches == [3]
    want = []
    for cs in sets:
        try:
            M.get_model(tuple(cs))
            want.append(True)
        except M.UnsatError:
            want.append(False)
    assert got == want
    assert got[1] is False                           # Python False short-circuits


def test_batch_is_possible_timeout_exhausted(batch_env):
    eng, z3_calls = batch_env
    M.time_handler.start_execution(0)
    assert M.batch_is_possible([(c_sat(),), (c_sat(),)]) == [False, False]
    assert eng.batches == [] and z3_calls == []


def test_filter_possible_keeps_order_and_states(batch_env):
    class S:
        def __init__(self, c):
            self.constraints = c
    states = [S((c_sat(),)), S((c_sat(), False)), S((True, c_sat()))]
    kept = M.filter_possible(states, constraints_of=lambda s: s.constraints)
    assert kept == [states[0], states[2]]


# ---- independence splitting ------------------------

def test_dependence_buckets_group_by_shared_symbols():
    from mythril_amd.smt import Array, Function
    bv = symbol_factory.BitVecSym
    x, y, z, w = bv("x", 256), bv("y", 256), bv("z", 256), bv("w", 256)
    a = Array("arr", 256, 256)
    f = Function("keccak256_256", 256, 256)
    cs = [x == symbol_factory.BitVecVal(1, 256),          # 0: {x}
          y == symbol_factory.BitVecVal(2, 256),          # 1: {y}
          (x + z) == symbol_factory.BitVecVal(3, 256),    # 2: {x, z} -> joins 0
          a[y] == symbol_factory.BitVecVal(4, 256),       # 3: {arr, y} -> joins 1
          f(w) == symbol_factory.BitVecVal(5, 256),       # 4: {f, w}
          f(z) == symbol_factory.BitVecVal(6, 256),       # 5: {f, z} -> joins 0 and 4
          symbol_factory.BitVecVal(1, 8) == symbol_factory.BitVecVal(1, 8)]   # 6: none
    raws = [c.raw for c in cs]
    groups = M.dependence_buckets(raws)
    as_idx = sorted(sorted(raws.index(c) for c in g) for g in groups)
    assert as_idx == [[0, 2, 4, 5], [1, 3], [6]]


def test_bucketed_witness_joins_group_assignments(monkeypatch, fresh):
    """gpu_search over independent groups: one batched search, the joint
    witness is the union of the group witnesses."""
    import numpy as np
    bv = symbol_factory.BitVecSym
    x, y = bv("x", 256), bv("y", 256)
    nodes = [(x == symbol_factory.BitVecVal(9, 256)).raw, (y == symbol_factory.BitVecVal(4, 256)).raw]

    class Eng:
        calls = 0

        def load(self, prog, leafgen, prog_seed=0):
            return prog

        def batch_search(self, loaded, seed, n_cand, first_index=0, want_probes=False):
            Eng.calls += 1
            out = []
            for p in loaded:
                w = np.zeros((len(p.leaves), 8), np.uint32)
                w[0, 0] = 9 if p.leaves[0].name == "x" else 4
                out.append((3, w))
            return out

        def witness(self, p, seed, index):
            # solve mode defines x / y by their equalities: the program
            # computes them (probes), as one re-evaluated lane would
            import ir_sim
            leaves = np.zeros((len(p.leaves), 8), np.uint32)
            _, probes = ir_sim.run(p, [0] * len(p.leaves))
            pr = np.zeros((len(probes), 8), np.uint32)
            for k, v in enumerate(probes):
                pr[k] = [(v >> (32 * j)) & 0xFFFFFFFF for j in range(8)]
            return leaves, pr
    monkeypatch.setattr(M, "get_engine", lambda dev=0, slot=0: Eng())
    a, progs = REAL_GPU_SEARCH(nodes, 200)
    assert Eng.calls == 1 and len(progs) == 2
    assert a.vars == {"x": 9, "y": 4}


# ---- failure handling, deadline, hand-over, statistics, Model (round 2) ----

@pytest.fixture
def reset_engine_memo():
    M._engine_failed = None
    M._batch_witness.clear()
    M._gpu_missed.clear()
    yield
    M._engine_failed = None
    M._batch_witness.clear()
    M._gpu_missed.clear()


def test_engine_init_failure_is_remembered(monkeypatch, fresh, reset_engine_memo):
    from mythril_amd.engine import EngineUnavailable
    calls = []

    def no_gpu(nodes, budget_ms):
        calls.append(1)
        raise EngineUnavailable("mg_init failed")
    monkeypatch.setattr(M, "gpu_search", no_gpu)
    x = symbol_factory.BitVecSym("x", 256)
    for k in range(3):
        with pytest.raises(M.SolverUnavailable):       # -> z3 (absent here)
            M.get_model((ULT(x, symbol_factory.BitVecVal(k + 5, 256)),))
    assert calls == [1]


def test_unexpected_prefilter_error_falls_back(monkeypatch, fresh, reset_engine_memo):
    def broken(nodes, budget_ms):
        raise AttributeError("bug in a front-end")
    monkeypatch.setattr(M, "gpu_search", broken)
    before = M.stats.errors
    with pytest.raises(M.SolverUnavailable):
        M.get_model((c_sat(),))
    assert M.stats.errors == before + 1


def test_gpu_miss_does_not_shorten_the_z3_timeout(monkeypatch, fresh, reset_engine_memo):
    """The fallback gets the reference's own timeout (support/model.py:26-31),
    whatever the GPU search took: a query z3 solves close to
    its timeout must not become unknown -> UnsatError because of a miss."""
    import time
    seen = {}

    def slow_miss(nodes, budget_ms):
        seen["budget"] = budget_ms
        time.sleep(0.15)
        return None

    def fake_z3(constraints, minimize, maximize, timeout):
        seen["z3_timeout"] = timeout
        raise M.UnsatError
    monkeypatch.setattr(M, "gpu_search", slow_miss)
    monkeypatch.setattr(M, "_z3_check", fake_z3)
    M.args.solver_timeout = 400
    with pytest.raises(M.UnsatError):
        M.get_model((c_sat(),))
    assert seen["budget"] <= 200
    assert seen["z3_timeout"] == 400


def test_fallback_is_capped_by_the_execution_time_left(monkeypatch, fresh, reset_engine_memo):
    """the fallback keeps the full solver timeout when time allows,
    but under enforce_execution_time it is capped by what is left of the
    execution time after the GPU phase (minus the reference's 500 ms), and
    no time left at that point raises UnsatError as at the entry."""
    import time
    seen = {}

    def slow_miss(nodes, budget_ms):
        time.sleep(0.3)
        return None

    def fake_z3(constraints, minimize, maximize, timeout):
        seen["z3_timeout"] = timeout
        raise M.UnsatError
    monkeypatch.setattr(M, "gpu_search", slow_miss)
    monkeypatch.setattr(M, "_z3_check", fake_z3)
    M.args.solver_timeout = 10000
    M.time_handler.start_execution(1.5)          # 1500 ms: 1000 ms budget at entry
    with pytest.raises(M.UnsatError):
        M.get_model((c_sat(),))
    assert 500 <= seen["z3_timeout"] <= 750       # 1500 - 300 (GPU) - 500, clock slack
    M.get_model.cache_clear()
    seen.clear()
    M.time_handler.start_execution(0.8)          # 300 ms at entry, none after the GPU
    with pytest.raises(M.UnsatError):
        M.get_model((c_sat(),))
    assert "z3_timeout" not in seen               # raised before asking z3
    M.get_model.cache_clear()
    seen.clear()
    M.time_handler.start_execution(0.8)
    with pytest.raises(M.UnsatError):             # enforce_execution_time=False: full timeout
        M.get_model((c_sat(),), enforce_execution_time=False)
    assert seen["z3_timeout"] == 10000


def test_superset_skip_needs_a_subset_searched_as_far(monkeypatch):
    """a miss recorded at a small candidate count (a batch) does
    not stop a full search of a superset group; one at >= the count does."""
    M.clear_search_memos()
    small, full = 1 << 16, M.SEARCH_CANDIDATES
    sub = frozenset({101, 102})
    sup = frozenset({101, 102, 103})
    M._note_miss(sub, small)
    assert not M._known_miss(sup, full)
    assert M._known_miss(sup, small)
    M._note_miss(sub, full)
    assert M._known_miss(sup, full)
    assert not M._known_miss(frozenset({101, 104}), small)      # not a superset
    M.clear_search_memos()


def test_batch_witness_is_handed_to_get_model(batch_env, monkeypatch, reset_engine_memo):
    eng, z3_calls = batch_env
    searches = []
    monkeypatch.setattr(M, "gpu_search", lambda nodes, budget_ms: searches.append(1))
    sat, unsat_like = (c_sat(),), (symbol_factory.Bool(False).__class__(symbol_factory.Bool(False).raw),)
    assert M.batch_is_possible([sat, unsat_like]) == [True, False]
    assert searches == []                        # neither set searched twice
    assert len(z3_calls) == 1                    # only the miss reached z3
    m = M.get_model(sat)                         # cached model of the batch witness
    assert m.assignment is not None and searches == []


def test_statistics_patch_extends_reference_repr():
    class RefStats:
        def __init__(self):
            self.query_count, self.solver_time = 3, 1.5

        def __repr__(self):
            return "Query count: {} \nSolver time: {}".format(self.query_count, self.solver_time)
    M._patch_statistics(RefStats)
    M._patch_statistics(RefStats)               # idempotent
    text = repr(RefStats())
    assert text.startswith("Query count: 3 \nSolver time: 1.5\nGPU pre-filter:")
    assert text.count("GPU pre-filter") == 1
    for phase in M.PHASES:
        assert phase in text


def test_model_getitem_follows_reference_semantics():
    class Z3Model:
        def __init__(self, d, size):
            self.d, self.size = d, size

        def __getitem__(self, item):
            if isinstance(item, int) and item >= self.size:
                raise IndexError(item)
            return self.d.get(item)

        def decls(self):
            return list(self.d)
    m = M.Model([Z3Model({"a": 1}, 1), Z3Model({"b": 2}, 1)])
    assert m["a"] == 1 and m["b"] == 2 and m["c"] is None
    with pytest.raises(IndexError):              # the last model's IndexError propagates
        m[5]
    assert M.Model([Z3Model({}, 0), Z3Model({"b": 2}, 3)])[1] is None   # earlier one skipped
    w = M.Model(None, Assignment(vars={"x": 7}))
    assert w["x"] == 7 and w["y"] is None


def test_env_configuration():
    saved = (M.GPU_ENABLED, list(M.DEVICES), M.SEARCH_CANDIDATES, M.SEARCH_BUDGET_MS)
    try:
        M.configure_from_env({"MYTHRIL_GPU": "0", "MYTHRIL_GPU_DEVICES": "0,2,3",
                              "MYTHRIL_GPU_CANDIDATES": "5000000", "MYTHRIL_GPU_BUDGET_MS": "50"})
        assert M.GPU_ENABLED is False and M.DEVICES == [0, 2, 3]
        assert M.SEARCH_CANDIDATES == 1 << 22 and M.SEARCH_BUDGET_MS == 50.0
        M.configure_from_env({})
        assert M.GPU_ENABLED is True
    finally:
        M.GPU_ENABLED, M.DEVICES, M.SEARCH_CANDIDATES, M.SEARCH_BUDGET_MS = saved


def test_gpu_disabled_goes_straight_to_z3(monkeypatch, fresh, reset_engine_memo):
    monkeypatch.setattr(M, "GPU_ENABLED", False)
    with pytest.raises(M.SolverUnavailable):
        M.get_model((c_sat(),))
    assert fresh == []


def test_batch_search_spreads_programs_over_devices(monkeypatch):
    """Corpus axis inside one process: LPT over instruction counts, one
    engine (context) per device, results back in program order."""
    import numpy as np
    from mythril_amd.ir import compile_constraints
    from mythril_amd.smt import node as N

    class DevEngine:
        def __init__(self, dev):
            self.dev, self.seen = dev, []

        def load(self, prog, leafgen, prog_seed=0):
            return prog

        def batch_search(self, loaded, seed, n_cand, first_index=0, want_probes=False):
            self.seen.extend(loaded)
            return [(self.dev * 1000 + p.n_ins, np.zeros((len(p.leaves), 8), np.uint32))
                    for p in loaded]
    engines = {d: DevEngine(d) for d in (0, 1, 2)}
    monkeypatch.setattr(M, "get_engine", lambda dev=0, slot=0: engines[dev])
    monkeypatch.setattr(M, "DEVICES", [0, 1, 2])
    x = N.bv_var("x", 256)
    progs = [compile_constraints([N.bv_cmp("bvult", N.bv_op("bvmul", *([x] * (k + 2))), x)])
             for k in range(7)]
    hits = M.batch_search_devices(progs, 1 << 16)
    assert len(hits) == len(progs)
    owner = {}
    for d, e in engines.items():
        for p in e.seen:
            owner[id(p)] = d
    assert sorted(len(e.seen) for e in engines.values()) != [0, 0, 7]
    for p, (idx, _) in zip(progs, hits):
        assert idx == owner[id(p)] * 1000 + p.n_ins       # each program answered by its device


# ---- round 3: assignment axis, group-miss memo, verification with z3 -------

class StreamEngine:
    """A device whose candidate stream satisfies the program at fixed indices
    (the same on every device: counter-based streams)."""

    def __init__(self, dev, sat, log):
        self.dev, self.sat, self.log = dev, sorted(sat), log

    def load(self, prog, leafgen, prog_seed=0):
        return prog

    def search(self, lp, seed, n_cand, first_index=0):
        import numpy as np
        self.log.append((self.dev, first_index, n_cand))
        for i in self.sat:
            if first_index <= i < first_index + n_cand:
                return i, np.zeros((len(lp.leaves), 8), np.uint32)
        return -1, None

    def witness(self, prog, seed, index):
        import numpy as np
        import ir_sim
        _, probes = ir_sim.run(prog, [0] * len(prog.leaves))
        pr = np.zeros((len(probes), 8), np.uint32)
        for k, v in enumerate(probes):
            pr[k] = [(v >> (32 * j)) & 0xFFFFFFFF for j in range(8)]
        return np.zeros((len(prog.leaves), 8), np.uint32), pr


@pytest.mark.parametrize("sat", [[137], [70000, 5000, 9000], [1 << 21], [], [0], [(1 << 22) - 1]])
@pytest.mark.parametrize("G", [2, 3, 8])
def test_assignment_axis_equals_single_device_sweep(monkeypatch, sat, G):
    """device g takes candidates [g*N/G, (g+1)*N/G); the host MIN
    over devices is the first index one device sweeping [0, N) finds."""
    from mythril_amd.ir import compile_constraints
    from mythril_amd.smt import node as N
    x = N.bv_var("x", 256)
    prog = compile_constraints([N.bv_cmp("bvult", x, N.bv_num(9, 256))])
    n = 1 << 22
    log = []
    one = StreamEngine(0, sat, log)
    want = one.search(prog, 0, n)[0]
    log.clear()
    engines = {d: StreamEngine(d, sat, log) for d in range(G)}
    monkeypatch.setattr(M, "get_engine", lambda dev=0, slot=0: engines[dev])
    idx, _ = M.search_assignment_axis(prog, n, list(range(G)))
    assert idx == want
    ranges = sorted((f, f + k) for _, f, k in log)
    assert ranges[0][0] == 0 and ranges[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))       # a partition
    assert sorted(d for d, _, _ in log) == list(range(G))


def test_single_group_query_uses_every_device(monkeypatch, fresh, reset_engine_memo):
    log = []
    engines = {d: StreamEngine(d, [3 << 17], log) for d in range(4)}
    monkeypatch.setattr(M, "get_engine", lambda dev=0, slot=0: engines[dev])
    monkeypatch.setattr(M, "DEVICES", [0, 1, 2, 3])
    M.clear_search_memos()
    x = symbol_factory.BitVecSym("ax", 256)
    hit = REAL_GPU_SEARCH([ULT(x, symbol_factory.BitVecVal(7, 256)).raw], 200)
    assert hit is not None
    assert sorted(d for d, _, _ in log) == [0, 1, 2, 3]


@pytest.fixture
def miss_engine(monkeypatch):
    log = []
    eng = StreamEngine(0, [], log)                       # never satisfied
    monkeypatch.setattr(M, "get_engine", lambda dev=0, slot=0: eng)
    monkeypatch.setattr(M, "DEVICES", [0])
    M.clear_search_memos()
    yield log
    M.clear_search_memos()


def test_group_miss_memo_skips_repeated_and_extended_groups(miss_engine, fresh,
                                                            reset_engine_memo):
    log = miss_engine
    x = symbol_factory.BitVecSym("mx", 256)
    c1 = (x * x == symbol_factory.BitVecVal(3, 256)).raw
    c2 = ULT(x, symbol_factory.BitVecVal(1000, 256)).raw
    before = M.stats.memo_misses
    assert REAL_GPU_SEARCH([c1], 200) is None
    assert len(log) == 1                                 # searched once
    assert REAL_GPU_SEARCH([c1], 200) is None            # same group: no search
    assert REAL_GPU_SEARCH([c1, c2], 200) is None        # extends the missed group
    assert len(log) == 1
    assert M.stats.memo_misses == before + 2
    y = symbol_factory.BitVecSym("my", 256)
    REAL_GPU_SEARCH([ULT(y, symbol_factory.BitVecVal(5, 256)).raw], 200)
    assert len(log) == 2                                 # an unrelated group is searched


def test_group_miss_at_fewer_candidates_is_searched_again(miss_engine, fresh, reset_engine_memo):
    log = miss_engine
    x = symbol_factory.BitVecSym("fx", 256)
    c1 = (x * x == symbol_factory.BitVecVal(3, 256)).raw
    prog = M._compile_search([c1])
    M._note_miss(prog.group_key, 1 << 16)                # e.g. a crowded batch
    assert REAL_GPU_SEARCH([c1], 200) is None
    assert len(log) == 1 and log[0][2] > (1 << 16)       # searched, with more candidates


def test_compile_gate_skips_queries_over_budget(miss_engine, fresh, reset_engine_memo):
    log = miss_engine
    x = symbol_factory.BitVecSym("gx", 256)
    c = (x * x == symbol_factory.BitVecVal(3, 256)).raw
    before = M.stats.gated
    assert REAL_GPU_SEARCH([c], 0.0001) is None
    assert M.stats.gated == before + 1 and log == []


def test_batch_miss_not_handed_over_when_under_searched(batch_env, monkeypatch,
                                                        reset_engine_memo):
    """a set the batch searched with fewer candidates than
    get_model would use is not sent to z3 unsearched."""
    eng, z3_calls = batch_env
    unsat_like = (symbol_factory.Bool(False).__class__(symbol_factory.Bool(False).raw),)
    monkeypatch.setattr(M, "_n_cand", lambda progs, budget: 1 << 16 if len(progs) > 1 else 1 << 20)
    M.batch_is_possible([unsat_like, (c_sat(),)])
    assert M._take(M._gpu_missed, unsat_like) is None


def test_node_witness_verified_by_z3_when_present(monkeypatch, fresh):
    """north_star: every GPU witness is re-verified by z3 before a model is
    returned — mirror DAG nodes too (through z3bridge.to_z3)."""
    seen = {}
    monkeypatch.setattr(M.z3bridge, "available", lambda: True)
    monkeypatch.setattr(M.z3bridge, "to_z3", lambda n, memo: ("z3", n.id))

    def verify(raws, assignment, timeout_ms):
        seen["raws"], seen["timeout"] = raws, timeout_ms
        return None                                     # z3 rejects it
    monkeypatch.setattr(M.z3bridge, "verify", verify)
    c = c_sat()
    before = M.stats.rejected
    assert M._accept([c], Assignment(vars={"x": 1}), None, 1234) is None
    assert seen["raws"] == [("z3", c.raw.id)] and seen["timeout"] == 1234
    assert M.stats.rejected == before + 1


# ---- round 3: adaptive per-shape gate ----------------------------------------

def _miss_query(k):
    """A fresh group (new symbol) of one fixed shape that the stub never
    satisfies: x_k * x_k == 3."""
    x = symbol_factory.BitVecSym("sg%d" % k, 256)
    return [(x * x == symbol_factory.BitVecVal(3, 256)).raw]


def test_shape_gate_skips_a_shape_that_keeps_missing(miss_engine, fresh, reset_engine_memo):
    log = miss_engine
    before = M.stats.shape_skipped
    for k in range(M.SHAPE_MIN):                       # learning: every query searched
        assert REAL_GPU_SEARCH(_miss_query(k), 200) is None
    assert len(log) == M.SHAPE_MIN
    searched = []
    for k in range(M.SHAPE_MIN, M.SHAPE_MIN + 2 * M.SHAPE_PROBE):
        n = len(log)
        assert REAL_GPU_SEARCH(_miss_query(k), 200) is None
        searched.append(len(log) > n)
    assert sum(searched) == 2                          # one probe per SHAPE_PROBE queries
    assert M.stats.shape_skipped == before + 2 * M.SHAPE_PROBE - 2
    # another shape is unaffected
    y = symbol_factory.BitVecSym("sgy", 256)
    n = len(log)
    REAL_GPU_SEARCH([ULT(y, symbol_factory.BitVecVal(5, 256)).raw], 200)
    assert len(log) == n + 1
    # cold runs forget the statistics; the switch turns the gate off
    M.clear_search_memos()
    n = len(log)
    REAL_GPU_SEARCH(_miss_query(999), 200)
    assert len(log) == n + 1


def test_shape_gate_keeps_searching_a_shape_that_hits(monkeypatch, fresh, reset_engine_memo):
    log = []
    engines = {0: StreamEngine(0, [5], log)}          # every program satisfied at index 5
    monkeypatch.setattr(M, "get_engine", lambda dev=0, slot=0: engines[dev])
    monkeypatch.setattr(M, "DEVICES", [0])
    M.clear_search_memos()
    for k in range(3 * M.SHAPE_MIN):
        x = symbol_factory.BitVecSym("sh%d" % k, 256)
        assert REAL_GPU_SEARCH([ULT(x, symbol_factory.BitVecVal(9, 256)).raw], 200) is not None
    assert len(log) == 3 * M.SHAPE_MIN
    M.clear_search_memos()


def test_shape_gate_switch(miss_engine, fresh, reset_engine_memo, monkeypatch):
    log = miss_engine
    M.configure_from_env({"MYTHRIL_GPU_ADAPTIVE": "0"})
    try:
        for k in range(M.SHAPE_MIN + M.SHAPE_PROBE):
            REAL_GPU_SEARCH(_miss_query(500 + k), 200)
        assert len(log) == M.SHAPE_MIN + M.SHAPE_PROBE
    finally:
        M.configure_from_env({})


def test_query_shape_abstracts_leaves_not_structure():
    a, b = symbol_factory.BitVecSym("qa", 256), symbol_factory.BitVecSym("qb", 256)
    c = symbol_factory.BitVecSym("qc", 8)
    s1 = M.query_shape(ULT(a + b, a).raw)
    s2 = M.query_shape(ULT(b + a, b).raw)
    assert s1 == s2
    assert M.query_shape(ULT(a * b, a).raw) != s1
    assert M.query_shape((c == symbol_factory.BitVecVal(1, 8)).raw) != \
        M.query_shape((a == symbol_factory.BitVecVal(1, 256)).raw)


def test_repeated_devices_get_their_own_contexts(monkeypatch):
    """DEVICES=[0, 0]: two host threads must not share one context (its
    workspace and stream serve one thread); the k-th repeat of a device is
    slot k (engine.device_slots), and batch_search_devices asks for each."""
    from mythril_amd.engine import device_slots
    from mythril_amd.ir import compile_constraints
    from mythril_amd.smt import node as N
    assert device_slots([0, 0, 1, 0]) == [(0, 0), (0, 1), (1, 0), (0, 2)]
    asked = []

    class Eng:
        def load(self, prog, leafgen, prog_seed=0):
            return prog

        def batch_search(self, loaded, seed, n_cand, first_index=0, want_probes=False):
            return [(-1, None) for _ in loaded]

    def ge(dev=0, slot=0):
        asked.append((dev, slot))
        return Eng()
    monkeypatch.setattr(M, "get_engine", ge)
    monkeypatch.setattr(M, "DEVICES", [0, 0])
    x = N.bv_var("x", 256)
    progs = [compile_constraints([N.bv_cmp("bvult", x, N.bv_num(k + 3, 256))]) for k in range(4)]
    M.batch_search_devices(progs, 1 << 16)
    assert sorted(set(asked)) == [(0, 0), (0, 1)]


_REAL_GPU_SEARCH = M.gpu_search


def test_constant_groups_are_answered_on_the_host(batch_env, monkeypatch):
    """A group the compiler folds to a constant root needs no launch
    (model._ground_value): true joins the witness as is, false sends the
    query to z3 without searching its other groups, and the false group is
    remembered as a miss at any depth."""
    eng, z3_calls = batch_env
    monkeypatch.setattr(M, "gpu_search", _REAL_GPU_SEARCH)
    M.clear_search_memos()
    x = symbol_factory.BitVecSym("gx", 256)
    y = symbol_factory.BitVecSym("gy", 256)
    t = symbol_factory.BitVecVal(3, 8) == symbol_factory.BitVecVal(3, 8)
    f = symbol_factory.BitVecVal(3, 8) == symbol_factory.BitVecVal(4, 8)
    live = ULT(x, symbol_factory.BitVecVal(5, 256))
    raws = M._raw_nodes([t, live])
    progs = [M._compile_search(b) for b in M.dependence_buckets(raws)]
    assert sorted(M._ground_value(p) is True for p in progs) == [False, True]
    M.stats.reset_gpu()
    M.get_model((t, live), enforce_execution_time=False)
    assert eng.batches == [1] and M.stats.ground_true == 1       # only the live group
    eng.batches.clear()
    with pytest.raises(M.UnsatError):
        M.get_model((f, ULT(y, symbol_factory.BitVecVal(9, 256))), enforce_execution_time=False)
    assert eng.batches == [] and M.stats.ground_false == 1 and len(z3_calls) == 1
    fkey = M._group_key(M.dependence_buckets(M._raw_nodes([f]))[0])
    assert M._group_miss[fkey] == M.GROUND_MISS


def test_batch_is_possible_notes_misses_only_for_groups_it_searched(batch_env, monkeypatch):
    """a set with a group folded to false launches
    nothing, so its live and constant-true sibling groups were never
    searched and must not enter the group-miss memo (a later query that
    shares them would skip its search); the false group itself is a miss at
    any depth."""
    eng, z3_calls = batch_env
    monkeypatch.setattr(M, "gpu_search", _REAL_GPU_SEARCH)
    M.clear_search_memos()
    bv = symbol_factory.BitVecVal
    x = symbol_factory.BitVecSym("bx", 256)
    t = bv(3, 8) == bv(3, 8)
    f = bv(3, 8) == bv(4, 8)
    live = ULT(x, bv(5, 256))
    assert M.batch_is_possible([(f, live, t)], enforce_execution_time=False) == [False]
    assert eng.batches == []
    fkey = M._group_key(M.dependence_buckets(M._raw_nodes([f]))[0])
    lkey = M._group_key(M.dependence_buckets(M._raw_nodes([live]))[0])
    tkey = M._group_key(M.dependence_buckets(M._raw_nodes([t]))[0])
    assert M._group_miss.get(fkey) == M.GROUND_MISS
    assert lkey not in M._group_miss and tkey not in M._group_miss
    # the live group alone is still searched (and found) afterwards
    assert M.batch_is_possible([(live,)], enforce_execution_time=False) == [True]
    assert eng.batches == [1]


def test_extra_context_failure_keeps_the_gpu_path(batch_env, monkeypatch):
    """with a device listed twice, failing to create its second
    context (slot 1) drops that repeat and falls back for the query; it does
    not disable the GPU path (only a slot-0 failure does)."""
    from mythril_amd.engine import EngineUnavailable
    monkeypatch.setattr(M, "DEVICES", [0, 0, 1])
    monkeypatch.setattr(M, "_engine_failed", None)
    assert M._engine_failure(EngineUnavailable("oom", slot=1, device=0), None) is None
    assert M.DEVICES == [0, 1]
    assert M._engine_failure(EngineUnavailable("no gpu", slot=0, device=0), None) == "no gpu"
