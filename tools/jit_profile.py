#!/usr/bin/env python3
"""Dynamic instruction counts of compiled programs per IR family, from the
instruction-level simulator (tests/asm_sim.py) running corpus DAGs in
generator mode: VALU / SALU / other per record of each family, so the JIT's
remaining overhead can be located without a GPU.
usage: tools/jit_profile.py [dag ids...]   (C2 corpus DAGs)
       tools/jit_profile.py c3 [unit ids...]   (bench units of c3 / c4 / c5)"""
import bisect
import collections
import functools
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import asm_sim  # noqa: E402
from mythril_amd import jit  # noqa: E402
from mythril_amd.corpus import make_dag  # noqa: E402
from mythril_amd.engine import default_leafgen  # noqa: E402
from mythril_amd.ir import compile_constraints  # noqa: E402

SEED = 0x6D797468
jit.program_asm = functools.partial(jit.program_asm, marks=True)
CNT = collections.defaultdict(collections.Counter)
OPS = collections.defaultdict(collections.Counter)
NREC = collections.Counter()
_step = asm_sim.Wave.step


def kind(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("s_waitcnt", "s_nop")):
        return "wait"
    if op.startswith(("s_branch", "s_cbranch", "s_setpc", "s_swappc", "s_getpc")):
        return "branch"
    if op.startswith("s_load"):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    return "vmem/lds"


def step(self, op, a, pc):
    if not hasattr(self, "_marks"):
        ms = sorted((i, l) for l, i in self.labels.items() if l.startswith((".Lmark_", ".Lbody_", ".Ljp0")))
        self._marks = ([i for i, _ in ms], [l for _, l in ms])
    idx, labs = self._marks
    k = bisect.bisect_right(idx, pc) - 1
    lab = labs[k] if k >= 0 else "interp"
    if lab.startswith(".Lmark_"):
        fam = lab.split("_")[2]
    elif lab.startswith(".Lbody_"):
        fam = "body_" + lab.split("_")[1]
    else:
        fam = "entry"
    if pc < idx[0] if idx else True:
        fam = "interp"
    CNT[fam][kind(op)] += 1
    OPS[fam][op] += 1
    return _step(self, op, a, pc)


asm_sim.Wave.step = step
args = sys.argv[1:]
workload = args.pop(0) if args and args[0].startswith("c") else "c2"
dags = [int(x) for x in args] or ([0, 1, 2, 3, 5, 8] if workload == "c2" else
                                  list(range(0, 64, 8)))
for d in dags:
    if workload == "c2":
        roots, _ = make_dag(d, SEED)
        prog = compile_constraints(roots)
    else:
        import bench
        prog = bench.compile_unit((workload, d))[1]
    for name, n in prog.stats["hist"].items():
        NREC[name] += n
    asm_sim.simulate(prog, gen=(SEED, d, 4096, default_leafgen(prog)), jit=True)
tot = collections.Counter()
for c in CNT.values():
    tot.update(c)
T = sum(NREC.values())
print("IR records %d; per record: %s" % (T, {k: round(v / T, 2) for k, v in tot.most_common()}))
for fam in sorted(CNT, key=lambda f: -sum(CNT[f].values())):
    c = CNT[fam]
    print("%-12s n %5d  all/IR %5.2f  %s" % (fam, NREC.get(fam, 0), sum(c.values()) / T,
                                            {k: round(v / T, 2) for k, v in c.most_common()}))
    top = [(o, round(v / T, 2)) for o, v in OPS[fam].most_common(8) if not o.startswith("v_")]
    print("             scalar/other top: %s" % top)
if os.environ.get("JIT_PROFILE_OP"):
    op = os.environ["JIT_PROFILE_OP"]
    print("\n%s per family (per IR record of the sample):" % op)
    for fam in sorted(OPS, key=lambda f: -OPS[f][op]):
        if OPS[fam][op]:
            print("  %-12s %6.2f" % (fam, OPS[fam][op] / T))
# measured SIMD cycles per wave64 instruction at 3 waves / SIMD
# (tools/valu_rate.hip, profiles/r03/valu_rate_r3*.log): plain VOP2 add/sub/
# logic/mov pair waves (2.67), everything else the kernel uses costs ~4
FAST = ("v_add_u32", "v_sub_u32", "v_subrev_u32", "v_and_b32", "v_or_b32", "v_xor_b32",
        "v_mov_b32", "v_not_b32")


def cycles(op):
    base = op.replace("_e32", "").replace("_e64", "")
    if base in FAST:
        return 2.67
    return 4.1


if os.environ.get("JIT_PROFILE_CYCLES"):
    cyc = {f: sum(cycles(o) * n for o, n in OPS[f].items() if o.startswith("v_")) for f in OPS}
    tot_c = sum(v for f, v in cyc.items() if f != "interp")
    print("\nVALU cycles per IR record by family (3 waves/SIMD rates), total %.1f:" % (tot_c / T))
    for f in sorted(cyc, key=lambda f: -cyc[f]):
        if f != "interp" and cyc[f]:
            top = sorted(((cycles(o) * n, o) for o, n in OPS[f].items() if o.startswith("v_")),
                         reverse=True)[:5]
            print("  %-12s %6.2f  %4.1f%%  %s" % (f, cyc[f] / T, 100 * cyc[f] / tot_c,
                                                 ", ".join("%s %.2f" % (o, c / T) for c, o in top)))
