#!/usr/bin/env python3
"""GPU triage of a compiled-program mismatch: for the given C2 DAG ids, the
program with every constraint probed runs on the interpreter and on its
compiled code over a lane range (mg_eval_gen: probes + generated leaves);
prints each differing lane and the constraints whose values differ, and
writes the compiled text to gpurun_out/jit_debug_<dag>.s."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from mythril_amd import jit  # noqa: E402
from mythril_amd.ir import compile_constraints  # noqa: E402

FIRST = (3 << 20) + 192
N = 4096
dags = [int(x) for x in sys.argv[1:]] or [7]
progs = []
for d in dags:
    roots = bench.workload_roots("c2", d)
    p = compile_constraints([], roots)
    progs.append((d, p))
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/jit_debug_%d.s" % d, "w") as fh:
        from mythril_amd.engine import default_leafgen as _lg
        fh.write("\n".join(jit.program_asm(p, _lg(p), d, ".Ljp0")))
images = {d: jit.compile_batch([(p, None, d)], workers=1) for d, p in progs}

from mythril_amd.engine import Engine, default_leafgen  # noqa: E402
eng = Engine(0)
for d, p in progs:
    lp = eng.load(p, default_leafgen(p), prog_seed=d)
    bi, pi, li = eng.eval_gen(lp, bench.SEED, FIRST, N, want_probes=True, want_leaves=True)
    h = eng.jit_attach([lp], images[d])
    bj, pj, lj = eng.eval_gen(lp, bench.SEED, FIRST, N, want_probes=True, want_leaves=True)
    eng.jit_detach(h)
    same = np.array_equal(pi, pj) and np.array_equal(li, lj)
    print("dag", d, "identical", same, flush=True)
    if not same:
        lanes = np.flatnonzero((pi != pj).any(axis=(0, 1)) | (li != lj).any(axis=(0, 1)))
        print("  lanes differing:", len(lanes), lanes[:16].tolist())
        for a in lanes[:4]:
            dif = [k for k in range(pi.shape[0]) if not np.array_equal(pi[k, :, a], pj[k, :, a])]
            print("  lane", int(a), "probes differing", dif[:12],
                  "leaves differ", bool((li[:, :, a] != lj[:, :, a]).any()))
            for k in dif[:3]:
                print("    probe", k, "interp", pi[k, :, a].tolist(), "jit", pj[k, :, a].tolist())
