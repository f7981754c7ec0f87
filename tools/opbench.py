#!/usr/bin/env python3
"""Per-opcode cost on the GPU: for each operator, a program of K dependent
instances (v = op(v, x[i % 4])) is evaluated under 2^20 generated
candidates; prints ns per instruction-lane and VALU cycles estimate."""

import json
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))

from mythril_amd.engine import get_engine
from mythril_amd.ir import compile_constraints
from mythril_amd.smt import node as N

K = 256
LANES = 1 << 20
BIN = ["bvadd", "bvsub", "bvmul", "bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod", "bvand",
       "bvor", "bvxor", "bvshl", "bvlshr", "bvashr"]


def chain(op):
    xs = [N.bv_var("x%d" % i, 256) for i in range(4)]
    v = xs[0]
    for i in range(K):
        if op in BIN:
            v = N.bv_op(op, v, xs[(i + 1) % 4])
        elif op == "eq":
            v = N.ite(N.eq(v, xs[(i + 1) % 4]), xs[i % 4], v)
        elif op == "ult":
            v = N.ite(N.bv_cmp("bvult", v, xs[(i + 1) % 4]), xs[i % 4], v)
        elif op == "extract":
            v = N.zero_extend(64, N.extract(200, 9, v))
        elif op == "concat":
            v = N.concat(N.extract(127, 0, v), N.extract(255, 128, xs[i % 4]))
        elif op == "umulno":
            v = N.ite(N.bv_cmp("bvumul_noovfl", v, xs[(i + 1) % 4]), xs[i % 4], v)
    return [N.bv_cmp("bvult", v, xs[0])]


def main():
    args = sys.argv[1:]
    lib = None
    if args and args[0].startswith("--lib="):
        lib = args.pop(0).split("=", 1)[1]
    from mythril_amd.engine import Engine
    eng = Engine(0, lib_path=__import__("os").path.abspath(lib)) if lib else get_engine(0)
    res = {}
    ops = args or BIN + ["eq", "ult", "extract", "concat", "umulno"]
    for op in ops:
        prog = compile_constraints(chain(op), nreg=eng.nreg)
        lp = eng.load(prog)
        eng.eval_gen(lp, 1, 0, LANES)
        t0 = time.perf_counter()
        reps = 3
        for r in range(reps):
            eng.eval_gen(lp, 1 + r, 0, LANES)
        dt = (time.perf_counter() - t0) / reps
        ns = dt * 1e9 / (prog.n_ins * LANES)
        # cycles per instruction per wave on one SIMD: CUs*4 SIMDs*2.4GHz / (lanes/64)
        cyc = dt * 2.4e9 * 256 * 4 / (prog.n_ins * LANES / 64)
        res[op] = {"n_ins": prog.n_ins, "ms": dt * 1e3, "ps_per_ins_lane": ns * 1e3,
                   "simd_cycles_per_wave_ins": cyc}
        print(op, json.dumps(res[op]), flush=True)


if __name__ == "__main__":
    main()
