"""Algorithmic work accounting for the constraint-node-evals/s metric.

Unit of work: one source-DAG node (after hash-consing CSE)
evaluated under one assignment.  The roofline is INT32 VALU: each node is
priced with a FIXED int32-op weight chosen independently of the
implementation (SURVEY.md §8d "Algorithmic work per unit"):

    ADD/SUB/NEG, AND/OR/XOR/NOT, EQ/DISTINCT/ULT/ULE/SLT/SLE(/GT/GE), BV ITE,
    CONCAT/EXTRACT/ZERO_EXT/SIGN_EXT                        8
    Bool and/or/xor/not/implies with k args                  max(1, k-1)
    SHL/LSHR/ASHR                                            24
    MUL                                                      192
    bvumul_noovfl                                            320
    UDIV/UREM/SDIV/SREM/SMOD                                 512
    SELECT over a store chain of length s                    8*s + 8
    free-array / UF lookup with e table entries              8*e + 8

A w-bit op scales by ceil(w/32)/8 (a 256-bit op is the unit).  Leaves
(variables, numerals, free and constant arrays) are not nodes; store nodes
are nodes of weight 0 (they are priced inside the selects that read them).

Round 5: work that is algorithmically cheaper than its
operator's generic weight is priced at what the cheaper algorithm costs, so
no workload's weighted ops exceed what an implementation must execute (C3
reported frac 1.054 under the generic weights):

    SHL/LSHR/ASHR by a constant amount                       8  (a funnel /
        bit-field extract per limb; SURVEY prices 24 for a VARIABLE amount)
    UDIV/UREM by a constant 2^k                              8  (the EXTRACT
        / shift they are: ir._Lowerer._by_constant)
    LASER's calldata word (calldata.py:47-54,219-232)
        Concat_{i<32} If(off+i <s size, select(cd, off+i), 0)
        over a free array with E model-table entries        16*E + 24
        (one 256-bit window compare + one 256-bit ITE per entry, the else
        broadcast, and the range mask as one compare + one ITE — the fused
        word of DESIGN §3.6 — instead of 32 table lookups, 32 signed
        compares, 32 ITEs, 31 index adds and a CONCAT); its byte terms, their
        compares, selects and index adds weigh 0 unless something other than
        a calldata word reads them.

Peak: the SIMD's int32 VALU issue capacity, MEASURED per SIMD
(``tools/valu_rate.hip``, ``profiles/r02/valu_rate.log``: every wave stamps
s_memtime and its HW_ID, and each SIMD's instructions are divided by the span
its waves covered, so co-residency is observed, not assumed).  Plain 32-bit
VALU (v_add_u32, v_xor_b32, v_add_f32) issues at 2.02 SIMD cycles per wave64
instruction with 8 waves per SIMD — MI355X_MICROARCH.md's "a wave64 VALU
instruction issues over 2 cycles" holds for int32 — while one wave alone
issues every 4.04 cycles (2.67 at 3 waves per SIMD, the interpreter's
occupancy).  64-bit-operand instructions (v_pk_mov_b32, v_mad_u64_u32,
v_pk_fma_f32) and carry chains (v_add_co / v_addc_co, carry through VCC) issue
at 4.0-4.1 cycles per SIMD at any occupancy.  The ceiling for int32 work is
therefore 256 CU x 4 SIMD x 64 lanes / 2.02 cycles x 2.4 GHz = 77.9 T
int32 lane-ops/s.  (Round 1 used a single wave's 4-cycle cadence, 38.4 T, as
the peak, which double-counted the fraction.)  A 256-bit ADD priced 8 ops is
8 carry-chain instructions at half rate, so the weighted-op definition above
cannot reach this ceiling for an add-heavy mix; it is the honest upper bound
for the int32 ops the weights count.
"""

from __future__ import annotations

from typing import Dict, Iterable, Tuple

from .smt.node import Node, topo_order

VALU_PEAK_OPS = 256 * 4 * 64 / 2.019 * 2.4e9  # measured int32 SIMD issue capacity (77.9 T)
HBM_PEAK_BPS = 8.0e12

_W8 = {"bvadd", "bvsub", "bvneg", "bvand", "bvor", "bvxor", "bvnot", "=", "distinct",
       "bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle", "bvsgt", "bvsge", "ite",
       "concat", "extract", "zero_extend", "sign_extend"}
_BOOL = {"and", "or", "xor", "not", "=>"}
_LEAF = {"var", "bvnum", "true", "false", "array", "K"}


def _scale(w: int) -> float:
    return ((w + 31) // 32) / 8.0


def node_weight(n: Node, table_sizes: Dict[str, int]) -> float:
    op = n.op
    if op in _LEAF or op == "store":
        return 0.0
    if n.is_bool() and op in _BOOL:
        return float(max(1, len(n.args) - 1))
    w = n.args[0].width if n.args and n.args[0].is_bv() else n.width
    if op in ("ite", "=", "distinct") and n.args and n.args[-1].is_bool():
        return 1.0
    if op in _W8:
        return 8.0 * _scale(max(w, n.width))
    if op in ("bvshl", "bvlshr", "bvashr"):
        if n.args[1].op == "bvnum":
            return 8.0 * _scale(w)             # constant amount: a bit-field move
        return 24.0 * _scale(w)
    if op == "bvmul":
        return 192.0 * _scale(w) * (len(n.args) - 1)
    if op == "bvumul_noovfl":
        return 320.0 * _scale(w)
    if op in ("bvudiv", "bvurem") and _pow2_divisor(n):
        return 8.0 * _scale(w)                 # x / 2^k, x % 2^k: an EXTRACT
    if op in ("bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod"):
        return 512.0 * _scale(w)
    if op == "select":
        s, a = 0, n.args[0]
        while a.op == "store":
            s, a = s + 1, a.args[0]
        extra = 8 * table_sizes.get(a.params[0], 2) + 8 if a.op == "array" else 0
        return 8.0 * s + 8.0 + extra
    if op == "apply":
        return 8.0 * table_sizes.get(n.params[0], 2) + 8.0
    return 8.0


def _pow2_divisor(n: Node) -> bool:
    d = n.args[1]
    return d.op == "bvnum" and d.params[0] > 0 and not d.params[0] & (d.params[0] - 1)


def _index_parts(x: Node):
    """(base, constant) with x = base + constant (mod 2^256), as
    ``ir._Lowerer._index_parts`` splits a calldata index."""
    c = 0
    while True:
        if x.op == "bvnum":
            return None, (c + x.params[0]) % (1 << 256)
        if x.op != "bvadd" or len(x.args) != 2:
            return x, c
        a, b = x.args
        if b.op == "bvnum" and a.op != "bvnum":
            x, c = a, (c + b.params[0]) % (1 << 256)
        elif a.op == "bvnum" and b.op != "bvnum":
            x, c = b, (c + a.params[0]) % (1 << 256)
        else:
            return x, c


def calldata_word(n: Node):
    """(array name, [nodes of the word's byte terms]) when ``n`` is LASER's
    calldata word over a free array — the shape ``ir._Lowerer._calldata_word``
    fuses (eval form) — else None.  The node list holds the 32 ITEs, their
    compares and selects, and the index terms of bytes 1..31 (byte 0's index
    is the offset, an operand of the fused word)."""
    if n.op != "concat" or n.width != 256 or len(n.args) != 32:
        return None
    size = arr = base = None
    c0 = 0
    inner = []
    for i, x in enumerate(n.args):
        if x.op != "ite" or x.width != 8:
            return None
        cond, sel, zero = x.args
        if zero.op != "bvnum" or zero.params[0] != 0 or cond.op != "bvslt" or sel.op != "select":
            return None
        idx = sel.args[1]
        if cond.args[0] is not idx or idx.width != 256:
            return None
        if i == 0:
            size, arr = cond.args[1], sel.args[0]
            if arr.op != "array":
                return None
            base, c0 = _index_parts(idx)
        elif cond.args[1] is not size or sel.args[0] is not arr:
            return None
        else:
            b, c = _index_parts(idx)
            if b is not base or c != (c0 + i) % (1 << 256):
                return None
            inner.append(idx)
        inner.extend((x, cond, sel))
    return arr.params[0], inner


def dag_work(roots: Iterable[Node], table_sizes: Dict[str, int] = None) -> Tuple[int, float]:
    """(node count, int32-op weight) of the DAG reachable from ``roots``.
    The node count is the metric's unit and does not depend on how a node is
    priced; the weight prices fused calldata words as one lookup each (module
    docstring) and their byte terms at 0 unless a non-word node reads them."""
    ts = table_sizes or {}
    order = topo_order(list(roots))
    users: Dict[int, list] = {}
    for n in order:
        for a in n.args:
            users.setdefault(a.id, []).append(n.id)
    words: Dict[int, float] = {}
    cand = set()
    for n in order:
        cw = calldata_word(n)
        if cw is not None:
            name, inner = cw
            words[n.id] = 16.0 * ts.get(name, 2) + 24.0
            cand.update(x.id for x in inner)
    # absorbed: every reader is a word or another absorbed term (readers come
    # later in topological order, so walk it backwards)
    absorbed = set()
    for n in reversed(order):
        if n.id in cand and all(u in words or u in absorbed for u in users.get(n.id, ())):
            absorbed.add(n.id)
    nodes = 0
    weight = 0.0
    for n in order:
        if n.op in _LEAF:
            continue
        nodes += 1
        if n.id in words:
            weight += words[n.id]
        elif n.id not in absorbed:
            weight += node_weight(n, ts)
    return nodes, weight
