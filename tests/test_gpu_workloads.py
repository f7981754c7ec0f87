"""GPU parity on the C1 / C3 / C4 stand-in query shapes
(mythril_amd/workloads.py) against oracle/evalref.c on every lane.

For 32 distinct queries per shape, in both table forms (leaf-keyed, as the
bench compiles them; constant-keyed with per-leaf pools, as the search
compiles them), the engine evaluates 4096 device-generated candidates; the
oracle evaluates the source DAG under the very leaves the engine generated
(checked against oracle/gen_ref.py on sampled lanes).  Every constraint's
value (a probe per constraint) and the root bit must match on every lane.
The witness search on the same shapes never returns a model the oracle
rejects."""

import os

import numpy as np
import pytest

from mythril_amd import workloads as W
from mythril_amd.assign import unpack
from mythril_amd.engine import default_leafgen, limbs_to_int
from mythril_amd.ir import compile_constraints
from mythril_amd.model import search_leafgen
from oracle import evalref, gen_ref
from oracle import smtlib_ref as R

pytestmark = pytest.mark.gpu
THREADS = int(os.environ.get("OMP_NUM_THREADS", "0")) or 8


# C1 (suicide.sol -t 2) has only ~20 distinct paths; C3 / C4 have hundreds
DISTINCT = {"c1": 16, "c3": 32, "c4": 32, "c5": 48}


def distinct_queries(name, k=None):
    k = k or DISTINCT[name]
    seen, out = set(), []
    for q in W.queries(name, 8 * k):
        key = tuple(c.id for c in q)
        if key not in seen:
            seen.add(key)
            out.append(q)
        if len(out) == k:
            break
    assert len(out) == k
    return out


def _table(prog):
    return [sum(int(prog.consts[i, j]) << (32 * j) for j in range(8))
            for i in range(prog.consts.shape[0])]


@pytest.mark.parametrize("const_keys", [False, True], ids=["leafkeyed", "constkeyed"])
@pytest.mark.parametrize("name", ["c1", "c3", "c4", "c5"])
def test_workload_every_lane_every_constraint(engine, name, const_keys):
    n, seed, first = 4096, 0x5EED, 3 << 20
    checked = 0
    for qi, q in enumerate(distinct_queries(name)):
        prog = compile_constraints(q, probes=q, const_keys=const_keys, leaf_pools=const_keys)
        lg = search_leafgen(prog) if const_keys else default_leafgen(prog)
        lp = engine.load(prog, lg, prog_seed=qi)
        bits, probes, leaves = engine.eval_gen(lp, seed, first, n, want_probes=True,
                                               want_leaves=True)
        S = evalref.serialize(q, prog)
        want = evalref.run_leaves_soa(S, prog, leaves, per_root=True, threads=THREADS)
        got = (probes[:, 0, :] & 1).astype(bool).T                  # (n, constraints)
        assert probes.shape[0] == len(q)
        bad = np.argwhere(got != want)
        assert bad.size == 0, (name, qi, bad[:4].tolist())
        assert np.array_equal(bits, want.all(axis=1)), (name, qi)
        # the engine's generator is the oracle's (sampled lanes)
        table = _table(prog)
        for a in (0, 1, 777, n - 1):
            for li, l in enumerate(prog.leaves):
                off, cnt = (prog.pool_ranges[li] if const_keys and prog.pool_ranges
                            else (0, len(prog.const_values)))
                pct = (20, 40, 60) if const_keys else (50, 70, 85)
                v = gen_ref.gen_leaf(seed, qi, li, first + a, l.width, table[off:off + cnt], pct=pct)
                assert limbs_to_int(leaves[li, :, a]) == v, (name, qi, a, li)
        checked += 1
    assert checked == DISTINCT[name]


@pytest.mark.parametrize("name", ["c3", "c4", "c5"])
def test_workload_batch_entry_point(engine, name):
    """``mg_batch_eval_gen`` (the path ``bench.py --workload`` times) over 32
    queries against ``evalref.run_gen`` (same generator, same pools)."""
    import ctypes as C
    from mythril_amd import shard
    from mythril_amd.engine import unpack_bits
    hip = C.CDLL("libamdhip64.so.7")
    qs = distinct_queries(name)
    progs = [compile_constraints(q) for q in qs]
    loaded = [engine.load(p, default_leafgen(p), prog_seed=i) for i, p in enumerate(progs)]
    batch = engine.batch_create(loaded)
    n, first, seed = 1 << 14, 1 << 20, 0x6D797468
    bits = np.zeros((len(progs), n // 64), dtype=np.uint64)
    firsts = np.full(len(progs), shard.NONE, dtype=np.int64)
    d_bits, d_first = C.c_void_p(), C.c_void_p()
    assert hip.hipMalloc(C.byref(d_bits), C.c_size_t(bits.nbytes)) == 0
    assert hip.hipMalloc(C.byref(d_first), C.c_size_t(firsts.nbytes)) == 0
    try:
        assert hip.hipMemcpy(d_first, firsts.ctypes.data_as(C.c_void_p),
                             C.c_size_t(firsts.nbytes), 1) == 0
        engine.batch_eval_gen(batch, seed, first, n, d_bits.value, d_first.value)
        assert hip.hipDeviceSynchronize() == 0
        assert hip.hipMemcpy(bits.ctypes.data_as(C.c_void_p), d_bits, C.c_size_t(bits.nbytes), 2) == 0
        assert hip.hipMemcpy(firsts.ctypes.data_as(C.c_void_p), d_first,
                             C.c_size_t(firsts.nbytes), 2) == 0
    finally:
        engine.batch_free(batch)
        hip.hipFree(d_bits)
        hip.hipFree(d_first)
    for k, (q, p) in enumerate(zip(qs, progs)):
        want = evalref.run_gen(evalref.serialize(q, p), p, seed, k, first, n, THREADS)
        assert np.array_equal(unpack_bits(bits[k], n), want), (name, k)
        hit = np.flatnonzero(want)
        assert firsts[k] == (first + int(hit[0]) if hit.size else shard.NONE), (name, k)


@pytest.mark.parametrize("name", ["c1", "c3", "c4", "c5"])
def test_workload_search_is_sound(engine, name):
    """Batched witness search over the shape's queries (the drop-in path of
    ``batch_is_possible``): every witness satisfies the query in the oracle."""
    from mythril_amd.model import _compile_search, batch_search_devices, dependence_buckets
    qs = distinct_queries(name)
    groups = [b for q in qs for b in dependence_buckets(q)]   # as get_model splits them
    progs = [_compile_search(b) for b in groups]
    hits = batch_search_devices(progs, 1 << 20)     # witnesses incl. computed values
    n_hit = 0
    for g, p, (idx, a) in zip(groups, progs, hits):
        if idx < 0:
            continue
        assert R.eval_constraints(g, R.Assignment(a.vars, a.arrays, a.funcs)) == 1, name
        n_hit += 1
    print("%s: %d/%d independent groups with a GPU witness" % (name, n_hit, len(groups)))
