"""The drop-in's multi-device code paths on real kernels, with
``DEVICES = [0, 0]``: two independent contexts on the one GPU of the box,
driven from two host threads exactly as two devices would be.

* corpus axis — ``batch_search_devices`` spreads a batch of search programs
  over the contexts by LPT: every program's first witness index and witness
  must equal the one-context batched search;
* assignment axis — ``search_assignment_axis`` splits one program's
  candidate range over the contexts: the joint first index and witness must
  equal a one-context sweep of the whole range.
"""

import numpy as np
import pytest

import mythril_amd.model as M
from mythril_amd import workloads as W
from mythril_amd.engine import EngineError, device_slots, get_engine

pytestmark = pytest.mark.gpu
N_CAND = 1 << 20


def _groups(name, n_queries):
    progs, seen = [], set()
    for q in W.queries(name, n_queries):
        for b in M.dependence_buckets(q):
            key = tuple(c.id for c in b)
            if key in seen:
                continue
            seen.add(key)
            try:
                progs.append(M._compile_search_uncached(b))
            except M.Unsupported:
                continue
    return progs


def _same(a, b):
    return (a is None and b is None) or (a.vars == b.vars and a.arrays == b.arrays and
                                         a.funcs == b.funcs)


@pytest.fixture
def two_contexts(monkeypatch):
    monkeypatch.setattr(M, "DEVICES", [0, 0])
    assert device_slots(M.DEVICES) == [(0, 0), (0, 1)]
    assert get_engine(0, 0) is not get_engine(0, 1)       # two contexts, one GPU
    yield


def test_corpus_axis_on_two_contexts_equals_one(engine, two_contexts, monkeypatch):
    progs = _groups("c4", 24) + _groups("c1", 12)
    assert len(progs) >= 8
    two = M.batch_search_devices(progs, N_CAND)
    monkeypatch.setattr(M, "DEVICES", [0])
    one = M.batch_search_devices(progs, N_CAND)
    assert [i for i, _ in two] == [i for i, _ in one]
    assert all(_same(a, b) for (_, a), (_, b) in zip(two, one))
    assert sum(i >= 0 for i, _ in one) >= 4              # the comparison covers hits


def test_assignment_axis_on_two_contexts_equals_one_sweep(engine, two_contexts):
    progs = [p for p in _groups("c4", 24) if not p.solved][:4] + _groups("c1", 6)[:2]
    n_hits = 0
    for prog in progs:
        joint = M.search_assignment_axis(prog, N_CAND, M.DEVICES)
        lp = engine.load(prog, M.search_leafgen(prog), prog_seed=0)
        i, leaves = engine.search(lp, M.SEARCH_SEED, N_CAND)
        assert joint[0] == i
        if i >= 0:
            n_hits += 1
            assert _same(joint[1], M._witness(engine, lp, (i, leaves)))
    assert n_hits >= 1


def test_get_model_with_two_contexts(engine, two_contexts):
    """get_model end to end on DEVICES=[0, 0]: a multi-group query (corpus
    axis) and the reference's x == 2 model test (one group: assignment
    axis) return the models the one-device path returns."""
    from mythril_amd.smt import symbol_factory
    x = symbol_factory.BitVecSym("x", 256)
    M.get_model.cache_clear()
    M.clear_search_memos()
    m = M.get_model((x == symbol_factory.BitVecVal(2, 256),))
    assert m.assignment.vars["x"] == 2
    q = W.queries("c4", 8)[3]
    M.get_model.cache_clear()
    try:
        m2 = M.get_model(tuple(q))
    except M.SolverUnavailable:
        m2 = None
    M.get_model.cache_clear()
    M.clear_search_memos()
    M.DEVICES = [0]
    try:
        m1 = M.get_model(tuple(q))
    except M.SolverUnavailable:
        m1 = None
    M.get_model.cache_clear()
    assert (m1 is None) == (m2 is None)
    if m1 is not None:
        assert _same(m1.assignment, m2.assignment)


def test_batch_eval_gen_sets_its_device_and_refuses_a_foreign_batch(engine, two_contexts):
    """mg_batch_eval_gen makes its context's device
    current like every other entry point, so a thread that last used another
    context (here the second slot, on another host thread) still launches on
    the right device and gets the one-context result; a batch created on one
    context and launched through the other is refused (MG_E_ARG)."""
    import ctypes as C
    import threading
    from mythril_amd.ir import compile_constraints
    from mythril_amd.corpus import make_dag
    hip = C.CDLL("libamdhip64.so.7", mode=C.RTLD_GLOBAL)
    e0, e1 = get_engine(0, 0), get_engine(0, 1)
    progs = [compile_constraints(make_dag(d)[0]) for d in (3, 17, 250)]
    n, words = 1 << 14, (1 << 14) // 64
    out = {}

    def run(eng, tag):
        loaded = [eng.load(p, prog_seed=k) for k, p in enumerate(progs)]
        d_bits = C.c_void_p()
        assert hip.hipMalloc(C.byref(d_bits), C.c_size_t(len(progs) * words * 8)) == 0
        try:
            b = eng.batch_create(loaded)
            try:
                hip.hipSetDevice(0)
                eng.batch_eval_gen(b, 0x5EED, 64, n, d_bits.value)
                hip.hipDeviceSynchronize()
                host = np.zeros(len(progs) * words, np.uint64)
                assert hip.hipMemcpy(host.ctypes.data_as(C.c_void_p), d_bits, C.c_size_t(host.nbytes), 2) == 0
                out[tag] = host
            finally:
                eng.batch_free(b)
        finally:
            hip.hipFree(d_bits)

    run(e0, "main")
    t = threading.Thread(target=run, args=(e1, "thread"))
    t.start()
    t.join()
    assert np.array_equal(out["main"], out["thread"])
    loaded = [e0.load(p) for p in progs]
    b = e0.batch_create(loaded)
    try:
        with pytest.raises(EngineError, match="another context"):
            e1.batch_eval_gen(b, 1, 0, 64)
    finally:
        e0.batch_free(b)
