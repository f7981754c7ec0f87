#!/usr/bin/env python3
"""A/B several builds of libmythgpu in ONE process (interleaved rounds, same
device), on the op microbenchmark programs and a corpus slice.
usage: python tools/ab.py lib1.so lib2.so ... [--ops bvand,bvudiv] [--dags 128]"""

import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mythril_amd.corpus import make_dag
from mythril_amd.engine import Engine
from mythril_amd.ir import compile_constraints
from mythril_amd.roofline import dag_work
from tools.opbench import chain


def timeit(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--ops", default="bvand,bvadd,bvmul,bvudiv,bvshl,eq,extract")
    ap.add_argument("--dags", type=int, default=256)
    ap.add_argument("--lanes-log2", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    engines = [Engine(0, lib_path=os.path.abspath(l)) for l in args.libs]
    lanes = 1 << args.lanes_log2
    dags = [make_dag(d)[0] for d in range(args.dags)]
    nodes = sum(dag_work(r)[0] for r in dags)
    loaded = []
    progs_by_nreg = {}
    for e in engines:
        if e.nreg not in progs_by_nreg:
            progs_by_nreg[e.nreg] = (
                {op: compile_constraints(chain(op), nreg=e.nreg) for op in args.ops.split(",") if op},
                [compile_constraints(r, nreg=e.nreg) for r in dags])
        progs, corpus = progs_by_nreg[e.nreg]
        lp = {op: e.load(p) for op, p in progs.items()}
        lc = [e.load(p, prog_seed=d) for d, p in enumerate(corpus)]
        loaded.append((e, lp, e.batch_create(lc), lc, progs))
    res = {}
    for rnd in range(args.rounds):
        for li, (e, lp, batch, _, progs) in enumerate(loaded):
            for op, h in lp.items():
                t = timeit(lambda: e.eval_gen(h, 1, 0, lanes), 3)
                res.setdefault((li, op), []).append(t * 1e9 / (progs[op].n_ins * lanes) * 1e3)

            def corpus_sync():
                e.batch_eval_gen(batch, 7, 0, 1 << 18)   # ctx stream (stream=None)
                e.eval_gen(lp[next(iter(lp))], 1, 0, 1)   # same stream: waits for it
            t = timeit(corpus_sync, 2)
            res.setdefault((li, "corpus"), []).append(nodes * (1 << 18) / t / 1e9)
    for (li, op), v in sorted(res.items(), key=lambda kv: (kv[0][1], kv[0][0])):
        unit = "Gnode-evals/s" if op == "corpus" else "ps/ins-lane"
        print("%-8s lib%d %-40s %8.3f (min %.3f max %.3f) %s" % (
            op, li, os.path.basename(args.libs[li]), statistics.median(v), min(v), max(v), unit))


if __name__ == "__main__":
    main()
