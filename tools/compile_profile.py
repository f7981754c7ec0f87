#!/usr/bin/env python3
"""Function-level profile of the native compiler on get_model's search
compiles (compile is 2.2 of 6.3 ms of a cold C3 query).

Writes every independent group of the first distinct queries of a stream as
tests/fuzz_compile.cpp corpus records (search form: leaf pools, constant
keys, solve, hints, ABI presets — what model._compile_search_uncached asks
for), builds that driver with ``-O2 -pg`` against csrc/mg_compile.cpp, runs
it with no mutations over the corpus repeated ``--reps`` times, and prints
the gprof flat profile's top lines plus the per-phase split the compiler
reports itself (program metadata ``t_us``).

Usage: python tools/compile_profile.py [--stream c3] [--queries 24] [--reps 20]
"""

import argparse
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stream", default="c3")
    ap.add_argument("--queries", type=int, default=24)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--graph", default="", help="write gprof's call graph here")
    ap.add_argument("--save", default="", help="also write the corpus (one copy) here")
    ap.add_argument("--time", action="store_true",
                    help="no profiler: build -O2 and print the wall time per query (best of 5)")
    args = ap.parse_args()
    import numpy as np
    import mythril_amd.model as M
    from mythril_amd import workloads as W
    from mythril_amd.ccompile import flatten
    from test_native_compiler import _corpus_record
    seen, recs, phases = set(), [], []
    for q in W.queries(args.stream, 8 * args.queries):
        key = tuple(c.id for c in q)
        if key in seen:
            continue
        seen.add(key)
        for b in M.dependence_buckets(M._raw_nodes(q)):
            recs.append(_corpus_record(flatten(b), True))
            try:
                phases.append(M._compile_search_uncached(b).compile_us)
            except M.Unsupported:
                pass
        if len(seen) >= args.queries:
            break
    ph = np.array([p for p in phases if p], dtype=float).sum(axis=0) / len(seen)
    names = ("decode", "lower", "solve", "sinks", "schedule", "allocate", "pools", "meta")
    print("per query (us):", ", ".join("%s %.0f" % kv for kv in zip(names, ph)),
          "total %.0f" % ph.sum())
    if args.save:
        with open(args.save, "wb") as fh:
            fh.write(b"".join(recs))
    with tempfile.TemporaryDirectory() as d:
        corpus = os.path.join(d, "corpus.bin")
        with open(corpus, "wb") as fh:
            fh.write(b"".join(recs) * args.reps)
        exe = os.path.join(d, "prof")
        if args.time:
            import time
            subprocess.run(["g++", "-std=c++17", "-O2", "-I" + os.path.join(ROOT, "include"),
                            os.path.join(ROOT, "tests", "fuzz_compile.cpp"),
                            os.path.join(ROOT, "mythril_amd", "csrc", "mg_compile.cpp"), "-o", exe],
                           check=True)
            import resource
            best = []
            for _ in range(5):
                u0 = resource.getrusage(resource.RUSAGE_CHILDREN).ru_utime
                subprocess.run([exe, corpus, "0"], cwd=d, check=True, capture_output=True)
                best.append(resource.getrusage(resource.RUSAGE_CHILDREN).ru_utime - u0)
            print("native compile: %.0f us user CPU per query (best of 5, %d queries x %d reps)"
                  % (min(best) * 1e6 / (len(seen) * args.reps), len(seen), args.reps))
            return
        subprocess.run(["g++", "-std=c++17", "-O2", "-pg", "-I" + os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tests", "fuzz_compile.cpp"),
                        os.path.join(ROOT, "mythril_amd", "csrc", "mg_compile.cpp"), "-o", exe],
                       check=True)
        subprocess.run([exe, corpus, "0"], cwd=d, check=True, capture_output=True)
        out = subprocess.run(["gprof", "-b", "-p", exe, os.path.join(d, "gmon.out")],
                             capture_output=True, text=True, check=True).stdout
        print("\n".join(out.splitlines()[:args.top + 5]))
        if args.graph:
            g = subprocess.run(["gprof", "-b", "-q", exe, os.path.join(d, "gmon.out")],
                               capture_output=True, text=True, check=True).stdout
            with open(args.graph, "w") as fh:
                fh.write(g)


if __name__ == "__main__":
    main()
