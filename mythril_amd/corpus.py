"""Synthetic constraint corpus (BASELINE config C2).

4096 random 256-bit BitVec DAGs (64..512 nodes each, uniform), built with the
SMT node API so the full host path (lowering, scheduling, allocation) runs on
them.  Operator mix, weighted to Mythril's lowering:

    ADD/SUB 20 %  AND/OR/XOR/NOT 15 %  EQ/ULT/ULE/SLT 20 %  ITE 10 %
    CONCAT/EXTRACT/ZERO_EXT 10 %  MUL 8 %  SHL/LSHR/ASHR 7 %
    UDIV/UREM/SDIV/SREM 5 %  bvumul_noovfl 2 %  SELECT-over-STORE (chain <= 8) 3 %

Leaves: 4-16 free 256-bit variables per DAG plus one free array.  Seed
0x6d797468 ("myth"); DAG d uses SplitMix64(seed ^ d).  Operands are drawn with
locality (mostly from the last few values), like LASER's path constraints,
which are trees over a few shared sub-terms.  Every node reaches the root:
values nobody consumed are compared with a neighbour and conjoined.
"""

from __future__ import annotations

from typing import List, Tuple

from .smt import node as N

SEED = 0x6D797468
M64 = (1 << 64) - 1

# op classes with their weights (percent)
_CLASSES = [("addsub", 20), ("logic", 15), ("cmp", 20), ("ite", 10), ("bits", 10),
            ("mul", 8), ("shift", 7), ("div", 5), ("umulno", 2), ("select", 3)]


class SplitMix64:
    def __init__(self, seed: int):
        self.s = seed & M64

    def next(self) -> int:
        self.s = (self.s + 0x9E3779B97F4A7C15) & M64
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        return z ^ (z >> 31)

    def below(self, n: int) -> int:
        return self.next() % n

    def u256(self) -> int:
        return self.next() | (self.next() << 64) | (self.next() << 128) | (self.next() << 192)


def dag_seed(seed: int, dag_id: int) -> int:
    return SplitMix64(seed ^ dag_id).next()


def dag_target_nodes(dag_id: int, seed: int = SEED) -> int:
    """The node count DAG ``dag_id`` is generated with (its first draw):
    the cost estimate the corpus-axis sharding balances on, known without
    building the DAG (mythril_amd.shard.lpt_assign)."""
    return 64 + SplitMix64(dag_seed(seed, dag_id)).below(449)


def make_dag(dag_id: int, seed: int = SEED, n_nodes: int = 0) -> Tuple[List[N.Node], int]:
    """Return (constraints, source node count) for DAG ``dag_id``, built in
    a fresh hash-consing scope: its compiled program is then the same in
    every process (constants shared with DAGs built earlier would otherwise
    carry older ids and move in the schedule)."""
    with N.fresh_scope():
        return _make_dag(dag_id, seed, n_nodes)


def _make_dag(dag_id: int, seed: int, n_nodes: int) -> Tuple[List[N.Node], int]:
    rng = SplitMix64(dag_seed(seed, dag_id))
    target = n_nodes or 64 + rng.below(449)
    n_vars = 4 + rng.below(13)
    vars_ = [N.bv_var("d%d_v%d" % (dag_id, i), 256) for i in range(n_vars)]
    consts = []
    for _ in range(2 + rng.below(5)):
        k = rng.below(4)
        v = [rng.u256(), rng.next(), rng.next() & 0xFFFFFFFF, (1 << (8 * (1 + rng.below(31)))) - 1][k]
        consts.append(N.bv_num(v, 256))
    array = N.array_var("d%d_A" % dag_id, 256, 256)
    bvs: List[N.Node] = list(vars_)
    bools: List[N.Node] = []
    used = set()
    created = set()

    def note(n: N.Node) -> N.Node:
        created.add(n.id)
        return n

    def pick() -> N.Node:
        r = rng.below(100)
        if r < 22:
            n = vars_[rng.below(len(vars_))]
        elif r < 30:
            n = consts[rng.below(len(consts))]
        else:
            n = bvs[len(bvs) - 1 - rng.below(min(len(bvs), 6))]
        used.add(n.id)
        return n

    def pick_bool() -> N.Node:
        if not bools:
            a, b = pick(), pick()
            bools.append(note(N.bv_cmp("bvult", a, b)))
        n = bools[len(bools) - 1 - rng.below(min(len(bools), 4))]
        used.add(n.id)
        return n

    roots: List[N.Node] = []

    def retire():
        """A value that leaves the operand window unused is compared with its
        neighbour right away (so it reaches the root without a long live
        range); a Bool that leaves the window unused becomes a constraint."""
        if len(bvs) > 6 + len(vars_):
            v = bvs[-7]
            if v.id not in used and v.id in created:
                used.add(v.id)
                bools.append(note(N.bv_cmp("bvule", v, bvs[-8])))
        if len(bools) > 4:
            b = bools[-5]
            if b.id not in used and b.id not in roots_seen:
                roots_seen.add(b.id)
                roots.append(b)

    roots_seen = set()
    weights = [w for _, w in _CLASSES]
    cum = [sum(weights[:i + 1]) for i in range(len(weights))]
    while len(created) < target:
        r = rng.below(100)
        cls = next(name for (name, _), c in zip(_CLASSES, cum) if r < c)
        if cls == "addsub":
            bvs.append(note(N.bv_op("bvadd" if rng.below(2) else "bvsub", pick(), pick())))
        elif cls == "logic":
            k = rng.below(10)
            if k < 3 and len(bools) >= 2:
                a, b = pick_bool(), pick_bool()
                bools.append(note(N.bool_op(["and", "or", "xor"][k], a, b)))
            elif k == 3:
                bvs.append(note(N.bv_op("bvnot", pick())))
            else:
                bvs.append(note(N.bv_op(["bvand", "bvor", "bvxor"][k % 3], pick(), pick())))
        elif cls == "cmp":
            op = ["=", "bvult", "bvule", "bvslt", "bvugt", "bvsle"][rng.below(6)]
            a, b = pick(), pick()
            bools.append(note(N.eq(a, b) if op == "=" else N.bv_cmp(op, a, b)))
        elif cls == "ite":
            c = pick_bool()
            bvs.append(note(N.ite(c, pick(), pick())))
        elif cls == "bits":
            x = pick()
            k = 8 * (1 + rng.below(31))
            lo = 8 * rng.below((256 - k) // 8 + 1)
            e = note(N.extract(lo + k - 1, lo, x))
            if rng.below(2):
                bvs.append(note(N.zero_extend(256 - k, e)))
            else:
                y = pick()
                bvs.append(note(N.concat(note(N.extract(255 - k, 0, y)), e)))
        elif cls == "mul":
            bvs.append(note(N.bv_op("bvmul", pick(), pick())))
        elif cls == "shift":
            op = ["bvshl", "bvlshr", "bvashr"][rng.below(3)]
            x = pick()
            if rng.below(2):
                amt = note(N.zero_extend(248, note(N.extract(7, 0, pick()))))
            else:
                amt = pick()
            bvs.append(note(N.bv_op(op, x, amt)))
        elif cls == "div":
            op = ["bvudiv", "bvurem", "bvsdiv", "bvsrem"][rng.below(4)]
            bvs.append(note(N.bv_op(op, pick(), pick())))
        elif cls == "umulno":
            bools.append(note(N.bv_cmp("bvumul_noovfl", pick(), pick())))
        else:  # select over a store chain
            arr = array if rng.below(2) else N.const_array(256, consts[0])
            for _ in range(1 + rng.below(8)):
                arr = note(N.store(arr, pick(), pick()))
            bvs.append(note(N.select(arr, pick())))
        retire()
    # everything reaches the root
    dangling = [b for b in bvs[-7:] if b.id not in used and b.id in created]
    for i in range(0, len(dangling), 2):
        a = dangling[i]
        b = dangling[i + 1] if i + 1 < len(dangling) else vars_[0]
        used.update((a.id, b.id))
        bools.append(note(N.bv_cmp("bvule", a, b)))
    roots += [b for b in bools if b.id not in used and b.id not in roots_seen]
    if not roots:
        roots = [bools[-1]]
    return roots, len(created)


def make_corpus(n_dags: int = 4096, seed: int = SEED):
    return [make_dag(d, seed) for d in range(n_dags)]
