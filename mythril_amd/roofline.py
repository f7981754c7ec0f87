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
        return 24.0 * _scale(w)
    if op == "bvmul":
        return 192.0 * _scale(w) * (len(n.args) - 1)
    if op == "bvumul_noovfl":
        return 320.0 * _scale(w)
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


def dag_work(roots: Iterable[Node], table_sizes: Dict[str, int] = None) -> Tuple[int, float]:
    """(node count, int32-op weight) of the DAG reachable from ``roots``."""
    ts = table_sizes or {}
    nodes = 0
    weight = 0.0
    for n in topo_order(list(roots)):
        if n.op in _LEAF:
            continue
        nodes += 1
        weight += node_weight(n, ts)
    return nodes, weight
