#!/usr/bin/env python3
"""Sweep: the native compiler (include/mythcc.h) against the Python
specification (ir.compile_constraints_py + solve.py) on many more inputs
than tests/test_native_compiler.py holds — C2 corpus DAGs [lo, hi) and the
first QUERIES C3 / C4 / C5 bench units in eval form, and every independent group of the C1 / C3 / C4 / C5 / c3o stand-in streams in
search form (solve + hints + ABI presets, and the plain search form).
Prints running (compiles, mismatches) per part; every program must be
identical.
usage: tools/compiler_equiv.py LO HI QUERIES [SEED]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from mythril_amd import ir  # noqa: E402
from mythril_amd.ccompile import compile_native  # noqa: E402
import mythril_amd.model as M  # noqa: E402
from test_native_compiler import _same  # noqa: E402

bad = n = 0


def both(name, cons, probes=(), **kw):
    global bad, n
    n += 1
    try:
        a = ir.compile_constraints_py(cons, probes, **kw)
    except ir.Unsupported as e:
        a = ("unsupported", str(e))
    try:
        b = compile_native(cons, probes, **kw)
    except ir.Unsupported as e:
        b = ("unsupported", str(e))
    if isinstance(a, tuple) or isinstance(b, tuple):
        if a != b:
            bad += 1
            print(name, "MISMATCH", a if isinstance(a, tuple) else "ok",
                  b if isinstance(b, tuple) else "ok")
        return
    try:
        _same(a, b)
    except AssertionError as e:
        bad += 1
        print(name, "MISMATCH", e)


def main():
    from mythril_amd import workloads as W
    from mythril_amd.corpus import make_dag
    lo, hi, nq = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    seed = int(sys.argv[4]) if len(sys.argv) > 4 else None
    for d in range(lo, hi):
        both("c2/%d" % d, make_dag(d)[0])
    print("c2 compiles %d mismatches %d" % (n, bad), flush=True)
    import bench
    for wl in ("c3", "c4", "c5"):                # the bench units, eval form
        for d in range(nq):
            both("%s-eval/%d" % (wl, d), bench.workload_roots(wl, d))
        print("%s eval compiles %d mismatches %d" % (wl, n, bad), flush=True)
    for wl in ("c1", "c3", "c4", "c5", "c3o"):
        for qi, q in enumerate(W.queries(wl, nq, seed=seed)):
            for bi, b in enumerate(M.dependence_buckets(q)):
                both("%s/%d/%d" % (wl, qi, bi), b, (), leaf_pools=True, const_keys=True,
                     solve=True, search_hints=True, abi_presets=True)
                both("%s/%d/%d-plain" % (wl, qi, bi), b, (), leaf_pools=True, const_keys=True,
                     search_hints=True)
        print("%s compiles %d mismatches %d" % (wl, n, bad), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
