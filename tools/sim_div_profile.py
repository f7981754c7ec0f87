"""VALU per region of the division body in the ISA simulator (labels are the
generator's local labels; counts are per executed division)."""
import collections
import sys

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import asm_sim  # noqa: E402
from mythril_amd.corpus import make_dag  # noqa: E402
from mythril_amd.engine import default_leafgen  # noqa: E402
from mythril_amd.ir import compile_constraints  # noqa: E402

SEED = 0x6D797468
valu = collections.Counter()
ndiv = [0]
orig_step = asm_sim.Wave.step
st = {"in": False, "reg": None}


def step(self, op, a, pc):
    lab = self._lab_at.get(pc)
    if lab:
        if lab.startswith(".Lbody_DIV"):
            st["in"], st["reg"] = True, "entry"
            ndiv[0] += 1
        elif lab.startswith(".Lh") or lab.startswith(".Lbody_"):
            st["in"] = False
        elif st["in"]:
            st["reg"] = lab.rstrip("0123456789_")
    if st["in"] and op.startswith("v_"):
        valu[st["reg"]] += 1
    return orig_step(self, op, a, pc)


asm_sim.Wave.step = step
orig_init = asm_sim.Wave.__init__


def init(self, *a, **k):
    orig_init(self, *a, **k)
    self._lab_at = {v: k for k, v in self.labels.items()}


asm_sim.Wave.__init__ = init
for d in [0, 1, 2, 3, 5, 8, 13, 21]:
    roots, _ = make_dag(d, SEED)
    prog = compile_constraints(roots)
    asm_sim.simulate(prog, gen=(SEED, d, 0, default_leafgen(prog)))
n = ndiv[0]
print("divisions", n, "VALU/div %.1f" % (sum(valu.values()) / n))
for k in sorted(valu, key=lambda k: -valu[k]):
    print("%-12s %6.1f" % (k, valu[k] / n))
