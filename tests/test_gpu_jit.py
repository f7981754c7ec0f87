"""Compiled programs (mythril_amd/jit.py) on the GPU beyond the bench entry
point: every path a compiled program can take inside the kernel must give
the interpreter's results bit for bit.

* host SoA assignments with every node probed (mg_eval: memory leaves and
  probe stores, the cold paths of the compiled code) over every
  ``dag_cases`` case;
* device-generated candidates with probes and the leaves written back
  (mg_eval_gen with ``leaves_out``: the witness-regeneration path);
* the witness search (mg_batch_search: early-exit waves, first-index
  reduction, regeneration) over search-form programs of the C1 / C4
  stand-in streams.

The interpreter itself is pinned to the oracle by tests/test_gpu_parity.py.
"""

import random

import numpy as np
import pytest

import dag_cases
import mythril_amd.model as M
from mythril_amd import jit, workloads as W
from mythril_amd.assign import Assignment as PAssignment, pack
from mythril_amd.corpus import make_dag
from mythril_amd.engine import default_leafgen
from mythril_amd.ir import compile_constraints

pytestmark = pytest.mark.gpu
CASES = dag_cases.named_cases()
SEED = 0x6D797468


def _image(items):
    return jit.compile_batch(items, workers=8, start="spawn")


def test_jit_eval_soa_every_case(engine):
    names = sorted(CASES)
    progs, inputs = [], []
    for name in names:
        constraints, probes, gen, tables = CASES[name]
        prog = compile_constraints(constraints, probes, table_sizes=tables)
        rng = random.Random(7000 + len(name))
        asgs = [gen(rng) for _ in range(333)]
        progs.append(prog)
        inputs.append(pack(prog, [PAssignment(a.vars, a.arrays, a.funcs) for a in asgs]))
    loaded = [engine.load(p) for p in progs]
    want = [engine.eval(lp, soa, want_probes=True) for lp, soa in zip(loaded, inputs)]
    h = engine.jit_attach(loaded, _image([(p, None, 0) for p in progs]))
    try:
        for name, lp, soa, (r_i, p_i) in zip(names, loaded, inputs, want):
            r_j, p_j = engine.eval(lp, soa, want_probes=True)
            assert np.array_equal(r_i, r_j), name
            assert np.array_equal(p_i, p_j), name
    finally:
        engine.jit_detach(h)


def test_jit_eval_gen_probes_and_leaves(engine):
    dags = list(range(12)) + [571]
    progs = [compile_constraints([], make_dag(d, SEED)[0]) for d in dags]
    loaded = [engine.load(p, default_leafgen(p), prog_seed=d) for d, p in zip(dags, progs)]
    first, n = (5 << 20) + 64, 2048
    want = [engine.eval_gen(lp, SEED, first, n, want_probes=True, want_leaves=True)
            for lp in loaded]
    h = engine.jit_attach(loaded, _image([(p, None, d) for d, p in zip(dags, progs)]))
    try:
        for d, lp, (r_i, p_i, l_i) in zip(dags, loaded, want):
            r_j, p_j, l_j = engine.eval_gen(lp, SEED, first, n, want_probes=True, want_leaves=True)
            assert np.array_equal(l_i, l_j), d
            assert np.array_equal(p_i, p_j), d
            assert np.array_equal(r_i, r_j), d
    finally:
        engine.jit_detach(h)


@pytest.mark.parametrize("shape", ["c1", "c4"])
def test_jit_batch_search_same_witnesses(engine, shape):
    progs = []
    for q in W.queries(shape, 12):
        for b in M.dependence_buckets(q):
            progs.append(M._compile_search(b))
    gens = [M.search_leafgen(p) for p in progs]
    n_cand = 1 << 18

    def run():
        loaded = [engine.load(p, g, prog_seed=0) for p, g in zip(progs, gens)]
        return loaded, engine.batch_search(loaded, M.SEARCH_SEED, n_cand)

    _, want = run()
    loaded, _ = run()
    h = engine.jit_attach(loaded, _image([(p, g, 0) for p, g in zip(progs, gens)]))
    try:
        got = engine.batch_search(loaded, M.SEARCH_SEED, n_cand)
    finally:
        engine.jit_detach(h)
    assert [i for i, _ in got] == [i for i, _ in want]
    for (i, lg), (_, lw) in zip(got, want):
        if i >= 0:
            assert np.array_equal(lg, lw)
    assert any(i >= 0 for i, _ in want), "no witness in the sample: the test checks nothing"
