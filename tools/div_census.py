#!/usr/bin/env python3
"""How often is a division's divisor short for a WHOLE wave?  (VERDICT r3
item 5: a wave-uniform short-division path pays only if every active lane's
divisor fits one or two 32-bit limbs.)

For bench units of a workload, the C oracle evaluates every node of the
source DAG under the device generator's candidates (generator v8: one class
per leaf per 64-index group, so a wave of 64 consecutive candidates shares
each leaf's class) and, for every UDIV/UREM/SDIV/SREM/SMOD and every wave,
records the widest divisor magnitude of the wave.  Prints one JSON line: the
fraction of (division, wave) pairs whose divisors all fit 32 / 64 bits, and
the share of divisions with a constant divisor.

With --lengths it also prints, per wave-wide divisor length in limbs (0 = every
divisor zero), how long the wave's longest dividend is.

Usage: python tools/div_census.py [--workload c2] [--units 64] [--waves 8] [--lengths]
"""

import argparse
import collections
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--units", type=int, default=64)
    ap.add_argument("--waves", type=int, default=8)
    ap.add_argument("--lengths", action="store_true")
    args = ap.parse_args()
    import bench
    from oracle import evalref, gen_ref
    E = evalref.E
    divs = {E[k] for k in ("UDIV", "UREM", "SDIV", "SREM", "SMOD")}
    signed = {E["SDIV"], E["SREM"], E["SMOD"]}
    n = 64 * args.waves
    first = 1 << 20
    tot = fit32 = fit64 = const = 0
    lengths = collections.defaultdict(collections.Counter)
    for d in range(args.units):
        d, prog, _, _ = bench.compile_unit((args.workload, d))
        roots = bench.workload_roots(args.workload, d)
        S = evalref.serialize(roots, prog)
        recs = [(i, r) for i, r in enumerate(S.recs) if r[0] in divs]
        if not recs:
            continue
        lvs = [[gen_ref.gen_leaf(bench.SEED, d, li, first + a, l.width, prog.const_values)
                for li, l in enumerate(prog.leaves)] for a in range(n)]
        _, vals = evalref.run_leaves(S, prog, lvs, want_nodes=True)
        for i, r in recs:
            b = r[3]
            if S.recs[b][0] == E["NUM"]:
                const += args.waves
                tot += args.waves
                continue
            w = r[1]
            for wv in range(args.waves):
                mx = 0
                for a in range(64 * wv, 64 * wv + 64):
                    x = evalref.node_value(vals, a, b)
                    if r[0] in signed and (x >> (w - 1)) & 1:
                        x = (1 << w) - x
                    mx = max(mx, x)
                tot += 1
                fit32 += mx < (1 << 32)
                fit64 += mx < (1 << 64)
                if args.lengths:
                    mu = max(evalref.node_value(vals, a, r[2]) for a in range(64 * wv, 64 * wv + 64))
                    lengths[(mx.bit_length() + 31) // 32][(mu.bit_length() + 31) // 32] += 1
    for nd in sorted(lengths):
        print("divisor limbs %d: dividend limbs %s" % (nd, dict(sorted(lengths[nd].items()))))
    print(json.dumps({"workload": args.workload, "units": args.units, "waves": args.waves,
                      "division_waves": tot, "const_divisor": const / max(tot, 1),
                      "all_lanes_fit32": fit32 / max(tot, 1), "all_lanes_fit64": fit64 / max(tot, 1)}))


if __name__ == "__main__":
    main()
