"""The native host compiler (include/mythcc.h, mythril_amd/csrc/mg_compile.cpp)
emits exactly the program the Python compiler (ir.compile_constraints_py +
solve.py, the specification) emits: same instructions, constant table,
leaves, pools, tables, derived values and statistics — on every named DAG
case, C2 corpus DAGs, and every independent group of the C1 / C3 / C4
stand-in query streams in both search (solve) and eval form.  CPU only."""

import ctypes
import os
import re

import numpy as np
import pytest

from mythril_amd import build, ir
from mythril_amd.ccompile import compile_native, load

HDR = os.path.join(build.ROOT, "include", "mythcc.h")


def _same(a, b):
    assert np.array_equal(a.code, b.code)
    assert np.array_equal(a.consts, b.consts)
    for f in ("const_values", "n_lds", "n_probes", "n_roots", "table_sizes", "table_kinds",
              "table_ckeys", "pool_ranges", "derived", "entry_keys", "n_user_probes", "stats"):
        assert getattr(a, f) == getattr(b, f), f
    assert a.leaves == b.leaves
    assert (a.presets is None) == (b.presets is None)
    if a.presets is not None:
        assert (a.presets.vars, a.presets.arrays) == (b.presets.vars, b.presets.arrays)


def _both(cons, probes=(), **kw):
    try:
        a = ir.compile_constraints_py(cons, probes, **kw)
    except ir.Unsupported as e:
        with pytest.raises(ir.Unsupported) as ei:
            compile_native(cons, probes, **kw)
        assert str(ei.value) == str(e)
        return None
    b = compile_native(cons, probes, **kw)
    _same(a, b)
    return b


def test_library_exports_every_declared_symbol():
    lib = load()
    names = sorted(set(re.findall(r"^\s*(?:int|void|const char\*|const uint32_t\*)\s+(mgc_\w+)\s*\(",
                                  open(HDR).read(), re.M)))
    assert len(names) == 7
    for n in names:
        assert hasattr(lib, n), n
    ops = lib.mgc_source_ops().decode().split("\n")
    assert ops[0] == "bvnum" and ops[-1] == "?"


def test_named_cases_identical():
    import dag_cases
    for name, (c, p, _, ts) in dag_cases.named_cases().items():
        _both(c, p, table_sizes=ts or None)
        _both(c, p, table_sizes=ts or None, leaf_pools=True, const_keys=True)


def test_corpus_dags_identical():
    from mythril_amd.corpus import make_dag
    for d in list(range(12)) + [571, 1000, 4095]:
        _both(make_dag(d)[0])


@pytest.mark.parametrize("workload", ["c1", "c3", "c4"])
def test_query_streams_identical(workload):
    """Every group get_model searches (solve mode, with the ABI presets and
    hints _compile_search_uncached adds) and its eval form."""
    from mythril_amd import workloads as W
    import mythril_amd.model as M
    n = presets = 0
    for q in W.queries(workload, 12):
        for b in M.dependence_buckets(q):
            p = _both(b, (), leaf_pools=True, const_keys=True, solve=True, search_hints=True,
                      abi_presets=True)
            presets += p is not None and p.presets is not None
            _both(b, (), leaf_pools=True, const_keys=True, search_hints=True)
            _both(b)
            n += 1
    assert n >= 12
    if workload == "c3":
        assert presets > 0          # BECToken batchTransfer reads _receivers at ABI offsets


def test_refused_commits_identical():
    """The construction's refusals (solve.Solver.run / _culprit, round 6):
    c3o queries whose groups needed a refused commit (7, 16) and a SafeMath
    check whose group is refused into a live program, in both compilers."""
    from mythril_amd import workloads as W
    import mythril_amd.model as M
    qs = [W.queries("c3o", 64)[i] for i in (7, 16)] + [W.queries("c3", 64)[0]]
    for q in qs:
        for b in M.dependence_buckets(q):
            _both(b, (), leaf_pools=True, const_keys=True, solve=True, search_hints=True,
                  abi_presets=True)


def test_stream_bench_units_identical():
    """The eval form of the C3 / C4 / C5 bench units (the gated schedule
    choice of round 6 picks per program)."""
    import bench
    for wl in ("c3", "c4", "c5"):
        for d in range(4):
            _both(bench.workload_roots(wl, d))


def test_unsupported_and_errors():
    from mythril_amd.smt import node as N
    x = N.bv_var("x", 300)
    y = N.bv_var("y", 300)
    with pytest.raises(ir.Unsupported):          # arithmetic on a 300-bit value
        compile_native([N.eq(N.bv_op("bvadd", x, y), x)])
    _both([N.eq(N.bv_op("bvadd", x, y), x)])
    a = N.array_var("A", 256, 256)
    with pytest.raises(ir.Unsupported):
        compile_native([N.eq(a, a)])


def test_leaf_remat_policies_identical():
    from mythril_amd.corpus import make_dag
    roots = make_dag(3)[0]
    saved = ir.LEAF_REMAT
    try:
        for pol in ("spill", "scratch", "scratch4", "always"):
            ir.LEAF_REMAT = pol
            _both(roots)
    finally:
        ir.LEAF_REMAT = saved


def test_malformed_input_is_an_error_not_a_crash():
    """Operands must precede their users: the C ABI checks indices."""
    from mythril_amd.ccompile import _Input
    lib = load()
    i32 = lambda *v: (ctypes.c_int32 * len(v))(*v)  # noqa: E731
    i64 = lambda *v: (ctypes.c_int64 * len(v))(*v)  # noqa: E731
    keep = dict(op=i32(3, 3), sort=i32(1, 1), width=i32(1, 1), dom=i32(0, 0), id=i64(1, 2),
                arg_off=i32(0, 1, 1), args=i32(1),          # node 0 names node 1 as operand
                p0=i64(0, 0), p1=i64(0, 0), str=i32(-1, -1), cval_off=i32(-1, -1), cons=i32(0))
    a = {k: ctypes.addressof(v) for k, v in keep.items()}
    inp = _Input(2, a["op"], a["sort"], a["width"], a["dom"], a["id"], a["arg_off"], a["args"],
                 a["p0"], a["p1"], a["str"], a["cval_off"], None, b"", 0, 1, a["cons"],
                 0, None, 0, None, None, 2, 16, 0, None, 0, 0, 0, 1, 2, 1)
    res = ctypes.c_void_p()
    assert lib.mgc_compile(ctypes.byref(inp), ctypes.byref(res)) == 2
    assert b"order" in lib.mgc_error(res)
    lib.mgc_free(res)


def test_c_abi_path_identical():
    """The plain C ABI (Python-flattened mgc_input over ctypes) and the
    CPython front-end compile the same program."""
    from mythril_amd.ccompile import compile_native_ctypes
    from mythril_amd import workloads as W
    import mythril_amd.model as M
    import dag_cases
    for name, (c, p, _, ts) in list(dag_cases.named_cases().items())[:6]:
        _same(compile_native(c, p, table_sizes=ts or None), compile_native_ctypes(c, p, table_sizes=ts or None))
    for q in W.queries("c4", 3):
        for b in M.dependence_buckets(q):
            kw = dict(leaf_pools=True, const_keys=True, solve=True, search_hints=True, abi_presets=True)
            _same(compile_native(b, (), **kw), compile_native_ctypes(b, (), **kw))


def test_native_buckets_match_the_python_partition():
    from mythril_amd import workloads as W
    import mythril_amd.model as M
    import dag_cases
    qs = [q for wl in ("c1", "c3", "c4") for q in W.queries(wl, 8)]
    qs += [c for c, _, _, _ in dag_cases.named_cases().values() if c]
    for q in qs:
        q = list(q) + list(q[:2])                 # repeated entries too
        got = M.dependence_buckets(q)
        want = M.dependence_buckets_py(q)
        assert [[c.id for c in g] for g in got] == [[c.id for c in g] for g in want]


def _corpus_record(f, solve):
    """One fuzz_compile.cpp corpus record of flatten()'s arrays."""
    import struct
    hdr = [f["n_nodes"], f["n_strings"], len(f["cons"]), len(f["probes"]), len(f["table_name"]),
           2, 16, len(f["extra"]) // 32, int(solve), int(solve), int(solve), 1, 2, 1, int(solve),
           int(solve), len(f["cval"]) // 4, len(f["strings"]), len(f["args"])]
    out = struct.pack("<19i", *hdr)
    for k in ("op", "sort", "width", "dom", "id", "arg_off", "args", "p0", "p1", "str", "cval_off"):
        out += f[k].tobytes()
    out += bytes(f["cval"]) + f["strings"]
    for k in ("cons", "probes", "table_name", "table_size"):
        out += f[k].tobytes()
    return out + bytes(f["extra"])


def test_mutated_inputs_under_asan_ubsan(tmp_path):
    """The C ABI checks every index and count: real DAGs compile, and
    thousands of mutations of them end in a status code — never in an
    out-of-bounds access or undefined behaviour (ASan + UBSan build)."""
    import json
    import shutil
    import subprocess
    from mythril_amd import workloads as W
    from mythril_amd.ccompile import flatten
    from mythril_amd.corpus import make_dag
    import dag_cases
    import mythril_amd.model as M
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    recs = []
    for c, p, _, ts in list(dag_cases.named_cases().values())[:8]:
        recs.append(_corpus_record(flatten(c, p, ts or None), False))
    recs.append(_corpus_record(flatten(make_dag(5)[0]), False))
    for wl in ("c1", "c3", "c4"):
        for b in M.dependence_buckets(W.queries(wl, 2)[1])[:2]:
            recs.append(_corpus_record(flatten(b), True))
    corpus = tmp_path / "corpus.bin"
    corpus.write_bytes(b"".join(recs))
    exe = str(tmp_path / "fuzz_compile")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
                    "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-static-libasan",
                    "-I" + os.path.join(build.ROOT, "include"),
                    os.path.join(build.ROOT, "tests", "fuzz_compile.cpp"),
                    os.path.join(build.ROOT, "mythril_amd", "csrc", "mg_compile.cpp"), "-o", exe],
                   check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, str(corpus), "150"], capture_output=True, text=True, env=env, timeout=900)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    st = json.loads(r.stdout.strip().splitlines()[-1])
    assert st["inputs"] == len(recs) and st["valid_ok"] == len(recs)
    assert st["mutated_error"] > 0 and st["mutated_ok"] > 0


def test_concurrent_compiles_agree():
    """The front-end releases the GIL during the compile: programs compiled
    on several threads at once equal the sequential ones."""
    import threading
    from mythril_amd.corpus import make_dag
    dags = [make_dag(d)[0] for d in range(6)]
    want = [compile_native(r) for r in dags]
    got = [None] * (4 * len(dags))
    errs = []

    def work(k):
        try:
            got[k] = compile_native(dags[k % len(dags)])
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    threads = [threading.Thread(target=work, args=(k,)) for k in range(len(got))]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert not errs
    for k, p in enumerate(got):
        _same(p, want[k % len(dags)])
