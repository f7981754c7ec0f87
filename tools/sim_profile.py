import sys, collections, re
sys.path.insert(0,'tests'); sys.path.insert(0,'.')
import asm_sim
from mythril_amd import asmgen
from mythril_amd.corpus import make_dag
from mythril_amd.engine import default_leafgen
from mythril_amd.ir import compile_constraints
# label -> family
fam = {}
for name in asmgen.AOPS:
    for var in range(asmgen.NVAR):
        for b in (0,1):
            fam[".Lh%d_0" % asmgen.hid(asmgen.AOP[name], var, b)] = name
ent = collections.Counter(); valu = collections.Counter(); salu = collections.Counter(); nins = collections.Counter()
orig_step = asm_sim.Wave.step
state = {"cur": "entry"}
def step(self, op, a, pc):
    lab = self._lab_at.get(pc)
    if lab:
        if lab in fam: state["cur"] = fam[lab]; ent[fam[lab]] += 1
        elif lab.startswith(".Lbody_"): state["cur"] = "body_" + lab.split("_")[1]; ent[state["cur"]] += 1
    c = state["cur"]
    if op.startswith("v_"): valu[c] += 1
    else: salu[c] += 1
    return orig_step(self, op, a, pc)
asm_sim.Wave.step = step
orig_init = asm_sim.Wave.__init__
def init(self, *a, **k):
    orig_init(self, *a, **k)
    self._lab_at = {v: k for k, v in self.labels.items()}
asm_sim.Wave.__init__ = init
SEED=0x6d797468
tot_ins = collections.Counter()
for d in [0, 1, 2, 3, 5, 8, 13, 21]:
    roots,_ = make_dag(d, SEED); prog = compile_constraints(roots)
    for i in range(prog.n_ins): tot_ins[asmgen.AOPS[0]] += 0
    h = prog.stats["hist"]
    for k, v in h.items(): nins[k] += v
    asm_sim.simulate(prog, gen=(SEED, d, 0, default_leafgen(prog)))
T = sum(nins.values())
print("IR ins", T, "VALU/ins %.1f SALU/ins %.1f" % (sum(valu.values())/T, sum(salu.values())/T))
for k in sorted(valu, key=lambda k: -valu[k]):
    print("%-12s VALU %6.2f/ins  SALU %5.2f/ins  per-exec VALU %6.1f  n %d" % (k, valu[k]/T, salu[k]/T, valu[k]/max(1,ent[k]), ent[k]))
