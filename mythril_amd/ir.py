"""Host compiler: ``get_model`` constraint DAG → mythgpu IR program.

Pipeline:

1. **Lowering** — SMT-LIB nodes (``mythril_amd.smt.node``) become kernel-level
   operations on values of width <= 256 (``LNode``), hash-consed so DAG sharing
   survives.  Rewrites:
   * n-ary ``bvadd/bvmul/bvand/bvor/bvxor/and/or`` → binary chains;
   * ``bvugt/bvuge/bvsgt/bvsge`` → swapped ``ult/ule/slt/sle``; ``=>`` →
     ``or(not a, b)``; ``distinct`` → ``not(=)``; ``zero_extend`` is free
     (values are kept canonical);
   * ``select`` over ``store`` chains → ``ite(i = j, v, ...)`` chains
     (``select(store(A,i,v),j) = ite(i=j, v, select(A,j))``), over ``K`` →
     the constant, over a free array or an uninterpreted-function application
     → an ite chain over the model's table entries, each entry a pair of leaf
     values (``name#k<e>``, ``name#v<e>``) plus ``name#else`` — exactly how a
     z3 model interprets arrays and functions (``laser/smt/model.py``);
   * values wider than 256 bits (Keccak inputs are 512-bit concats,
     ``instructions.py:1029-1035``) are split into 256-bit chunks: only
     concat / extract / zero_extend / = / distinct / ite / table keys are
     supported on them, which is every use LASER makes of them;
   * the carry test z3 builds for ``BVAddNoOverflow``
     (``extract(w, w, bvadd(zext1 a, zext1 b))``) becomes ``ult(a+b, a)``.
   Anything else raises :class:`Unsupported` (the caller falls back to z3).
2. **Scheduling** — source creation order (topological, short live ranges),
   each sink (``ROOT`` per constraint, ``OUT`` per probe) right after its
   operand.
3. **Register allocation** — linear scan over 15 VGPR slots with Belady
   eviction (furthest next use); evicted values go to LDS (``SPILL`` /
   ``RELOAD``), constants are rematerialised.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import irdefs as I
from .smt.node import Node, topo_order

CHUNK = 256
MAX_SPILL = I.MAX_LDS + I.MAX_PSLOTS   # LDS tier first, then per-lane scratch
LDS_TIER = 6           # spill slots the assembly kernel keeps in LDS (mg_api.cpp)
# Leaf eviction policy: "spill" (a leaf is spilled like any value), "scratch"
# (a leaf that would need a per-lane scratch slot is regenerated at its next
# use instead), "scratchK" (regenerated unless one of the first K scratch
# slots is free), "always" (leaves are never spilled).  Regeneration costs
# the generator's VALU; a scratch spill costs HBM traffic.  Default
# "scratch2": with the round-2 generator (49 VALU per leaf) as fast as
# "scratch4" and "scratch6"/LDS-only slower (profiles/r02/remat_final/),
# at well under half the HBM traffic.
import os as _os
LEAF_REMAT = _os.environ.get("MYTHRIL_GPU_LEAF_REMAT", "scratch2")


class Unsupported(Exception):
    """The DAG uses something the GPU path does not evaluate (→ z3)."""


class LNode:
    __slots__ = ("op", "width", "args", "imm", "id", "birth")

    def __init__(self, op, width, args, imm, nid, birth):
        self.op = op
        self.width = width
        self.args = args
        self.imm = imm
        self.id = nid
        self.birth = birth     # id of the source node being lowered at creation

    def __repr__(self):
        return "L%d:%s/%d%s" % (self.id, I.OPNAME.get(self.op, self.op), self.width,
                                 "" if self.imm is None else "[%s]" % (self.imm,))


@dataclass
class Leaf:
    """One input slot of an assignment.  ``kind``: var | key | val | else |
    cval | aux (a search-mode selector, ``solve.py``, not part of a model);
    ``source`` is the variable / array / function name, ``chunk`` the 256-bit
    chunk of a wide value, ``entry`` the table entry index."""
    name: str
    width: int
    kind: str
    source: str
    chunk: int = 0
    entry: int = 0


@dataclass
class Program:
    code: np.ndarray                  # (n_ins, 4) uint32
    consts: np.ndarray                # (n_consts, 8) uint32
    const_values: List[int]
    leaves: List[Leaf]
    n_lds: int
    n_probes: int
    n_roots: int
    table_sizes: Dict[str, int]
    table_kinds: Dict[str, str] = field(default_factory=dict)   # name -> array | func
    # per table: the constant keys it is read at (compiled with const_keys);
    # entry i of the model is (table_ckeys[name][i], leaf "name#c<i>"), in
    # front of the table_sizes[name] leaf-keyed entries
    table_ckeys: Dict[str, List[int]] = field(default_factory=dict)
    stats: Dict[str, object] = field(default_factory=dict)
    # per-leaf (offset, count) of its candidate pool in the device constant
    # table (consts); empty unless compiled with leaf_pools
    pool_ranges: List[Tuple[int, int]] = field(default_factory=list)
    # solve mode: model values the program COMPUTES, reported as probe
    # chunks after the caller's probes — leaves defined by an equality
    # (leaf index -> probe index) and the keys of argument-keyed table
    # entries (table -> entry -> probe index per 256-bit key chunk)
    derived: Dict[int, int] = field(default_factory=dict)
    entry_keys: Dict[str, List[List[int]]] = field(default_factory=dict)
    n_user_probes: int = 0
    # search mode: fixed parts of every candidate model (abi.Plan: the ABI
    # offset words and calldatasize the query was compiled under)
    presets: object = None
    # search mode: the independent group's constraint node ids (model.py's
    # group-miss memo)
    group_key: object = None
    # register slots of the layout it was compiled for (16, or 11: the
    # four-wave layout); a context of that layout loads it (Engine.load)
    nreg: int = 16

    @property
    def solved(self) -> bool:
        """Witnesses need the probe values too (``assign.unpack``)."""
        return bool(self.derived or self.entry_keys or self.presets)

    @property
    def n_ins(self) -> int:
        return int(self.code.shape[0])

    def leaf_index(self) -> Dict[str, int]:
        return {l.name: i for i, l in enumerate(self.leaves)}


# ----------------------------------------------------------------------------
# lowering
# ----------------------------------------------------------------------------

def _limbs(value: int) -> List[int]:
    return [(value >> (32 * j)) & 0xFFFFFFFF for j in range(8)]


class _Lowerer:
    def __init__(self, table_sizes: Dict[str, int], default_entries: int):
        self.table = {}
        self.nid = 0
        self.leaves: List[Leaf] = []
        self.leaf_ids: Dict[str, int] = {}
        self.memo: Dict[int, List[LNode]] = {}
        self.sel_memo: Dict[Tuple[int, Tuple[int, ...]], List[LNode]] = {}
        self.table_sizes = dict(table_sizes)
        self.table_kinds: Dict[str, str] = {}
        self.default_entries = default_entries
        self.consts_seen: set = set()
        self.birth = 0
        self.table_ckeys: Dict[str, List[int]] = {}
        # solve mode (search): argument-keyed table entries, in lookup order
        self.solve = False
        self.solve_tables: set = set()
        self.arg_entries: Dict[str, List[Tuple[List[LNode], List[LNode]]]] = {}

    # -- hash-consed constructors ------------------------------------------
    def mk(self, op: int, width: int, args=(), imm=None) -> LNode:
        if op == I.CONCAT and width == I.MAX_WIDTH and args[0].op == I.EXTRACT and \
                args[0].imm == 0 and args[0].args[0].width == I.MAX_WIDTH:
            # concat(y[h:0], e) at 256 bits = (y << |e|) | e mod 2^256: the
            # funnel shift drops y's high bits itself (no EXTRACT needed)
            args = (args[0].args[0],) + tuple(args[1:])
        key = (op, width, tuple(a.id for a in args), imm)
        n = self.table.get(key)
        if n is None:
            self.nid += 1
            birth = self.birth
            for a in args:          # keep (birth, id) order topological
                if a.birth > birth:
                    birth = a.birth
            n = LNode(op, width, tuple(args), imm, self.nid, birth)
            self.table[key] = n
        return n

    def const(self, value: int, width: int) -> LNode:
        value &= (1 << width) - 1
        self.consts_seen.add(value)
        return self.mk(I.CONST, width, (), value)

    def leaf(self, name: str, width: int, kind: str, source: str, chunk=0, entry=0) -> LNode:
        idx = self.leaf_ids.get(name)
        if idx is None:
            idx = len(self.leaves)
            self.leaf_ids[name] = idx
            self.leaves.append(Leaf(name, width, kind, source, chunk, entry))
        return self.mk(I.LEAF, width, (), idx)

    # -- chunk helpers --------------------------------------------------------
    @staticmethod
    def nchunks(w: int) -> int:
        return (w + CHUNK - 1) // CHUNK

    @staticmethod
    def chunk_width(w: int, i: int) -> int:
        return min(CHUNK, w - CHUNK * i)

    def bits(self, chunks: Sequence[LNode], w: int, lo: int, hi: int) -> LNode:
        """Bits [lo, hi] (inclusive) of a chunked value, hi - lo < 256."""
        ci, cj = lo // CHUNK, hi // CHUNK
        if ci == cj:
            c = chunks[ci]
            cw = self.chunk_width(w, ci)
            l0, h0 = lo - CHUNK * ci, hi - CHUNK * ci
            if l0 == 0 and h0 == cw - 1:
                return c
            return self.mk(I.EXTRACT, h0 - l0 + 1, (c,), l0)
        low_w = CHUNK * (ci + 1) - lo
        low = self.bits(chunks, w, lo, CHUNK * (ci + 1) - 1)
        high = self.bits(chunks, w, CHUNK * cj, hi)
        return self.mk(I.CONCAT, hi - lo + 1, (high, low), low_w)

    def assemble(self, pieces: List[Tuple[List[LNode], int]]) -> List[LNode]:
        """Concatenate (chunks, width) pieces given MSB first."""
        total = sum(w for _, w in pieces)
        # segments LSB first: (chunks, width, offset in result)
        segs, off = [], 0
        for ch, w in reversed(pieces):
            segs.append((ch, w, off))
            off += w
        out = []
        for k in range(self.nchunks(total)):
            lo_k, hi_k = CHUNK * k, min(total, CHUNK * (k + 1)) - 1
            acc: Optional[LNode] = None
            acc_w = 0
            for ch, w, o in segs:
                a, b = max(lo_k, o), min(hi_k, o + w - 1)
                if a > b:
                    continue
                part = self.bits(ch, w, a - o, b - o)
                pw = b - a + 1
                if acc is None:
                    acc, acc_w = part, pw
                else:
                    acc = self.mk(I.CONCAT, acc_w + pw, (part, acc), acc_w)
                    acc_w += pw
            out.append(acc)
        return out

    # -- main lowering ---------------------------------------------------------
    def lower(self, n: Node) -> List[LNode]:
        r = self.memo.get(n.id)
        if r is not None:
            return r
        # iterative post-order so deep DAGs do not hit the recursion limit
        nodes = self._pending(n)
        skip = set()
        for m in nodes:            # operands consumed only through the carry pattern
            if m.op == "extract" and self._is_carry(m):
                s = m.args[0]
                skip.update((s.id, s.args[0].id, s.args[1].id))
        saved = self.birth
        for m in nodes:
            if m.id in self.memo or m.is_array() or (m.id in skip and m is not n):
                continue
            try:
                self.birth = m.id
                self.memo[m.id] = self._lower_one(m)
            except KeyError as e:   # a skipped operand was needed elsewhere
                raise Unsupported("operand lowered only as part of a pattern") from e
            finally:
                self.birth = m.id
        self.birth = max(saved, self.birth) if saved else self.birth
        return self.memo[n.id]

    def _pending(self, n: Node) -> List[Node]:
        """Post-order of the nodes under ``n`` not lowered yet: a lowered
        node's operands are not walked again (every constraint's lower()
        call walked the whole DAG below it; a carry pattern's skipped
        operands under a node lowered by an earlier call are then no longer
        in this call's skip set, so a later use elsewhere is lowered instead
        of being refused)."""
        memo, seen, out = self.memo, set(), []
        stack = [(n, False)]
        while stack:
            m, done = stack.pop()
            if done:
                out.append(m)
                continue
            if m.id in seen or m.id in memo:
                continue
            seen.add(m.id)
            stack.append((m, True))
            for a in reversed(m.args):
                if a.id not in seen and a.id not in memo:
                    stack.append((a, False))
        return out

    def _narrow(self, n: Node) -> LNode:
        ch = self.memo[n.id]
        if len(ch) != 1:
            raise Unsupported("%s on a %d-bit value" % (n.op, n.width))
        return ch[0]

    def _fold(self, op: int, width: int, args: List[LNode]) -> LNode:
        acc = args[0]
        for a in args[1:]:
            acc = self.mk(op, width, (acc, a))
        return acc

    def _by_constant(self, op: str, w: int, n: Node) -> Optional[LNode]:
        """Shifts by a constant and unsigned division / remainder by a power
        of two as bit-field ops (EVM SHR/SHL/SAR and DIV/MOD by 2^k keep
        their constant operand after z3's simplify): funnel EXTRACT /
        CONCAT / SEXT instead of the variable-shift and division bodies."""
        if n.args[1].op != "bvnum":
            return None
        c = n.args[1].params[0]
        x = self._narrow(n.args[0])
        if op in ("bvudiv", "bvurem"):
            if c <= 0 or c & (c - 1):
                return None
            k = c.bit_length() - 1
            if op == "bvurem":
                return self.const(0, w) if k == 0 else self.mk(I.EXTRACT, k, (x,), 0)
            op, c = "bvlshr", k
        if op not in ("bvshl", "bvlshr", "bvashr"):
            return None
        if c == 0:
            return x
        if op == "bvashr":
            c = min(c, w - 1)                     # >= w: every bit is the sign
            return self.mk(I.SEXT, w, (self.mk(I.EXTRACT, w - c, (x,), c),), w - c)
        if c >= w:
            return self.const(0, w)
        if op == "bvlshr":
            return self.mk(I.EXTRACT, w - c, (x,), c)
        return self.mk(I.CONCAT, w, (self.mk(I.EXTRACT, w - c, (x,), 0), self.const(0, c)), c)

    def _lower_one(self, n: Node) -> List[LNode]:
        op, w = n.op, n.width
        if w > CHUNK:
            return self._lower_wide(n)
        A = lambda i: self._narrow(n.args[i])  # noqa: E731
        if op == "bvnum":
            return [self.const(n.params[0], w)]
        if op == "true":
            return [self.const(1, 1)]
        if op == "false":
            return [self.const(0, 1)]
        if op == "var":
            return [self.leaf(n.params[0], w, "var", n.params[0])]
        simple = {"bvsub": I.SUB, "bvudiv": I.UDIV, "bvurem": I.UREM, "bvsdiv": I.SDIV,
                  "bvsrem": I.SREM, "bvsmod": I.SMOD, "bvshl": I.SHL, "bvlshr": I.LSHR,
                  "bvashr": I.ASHR}
        if op in simple:
            red = self._by_constant(op, w, n)
            if red is not None:
                return [red]
            return [self.mk(simple[op], w, (A(0), A(1)))]
        nary = {"bvadd": I.ADD, "bvmul": I.MUL, "bvand": I.AND, "bvor": I.OR, "bvxor": I.XOR,
                "and": I.AND, "or": I.OR}
        if op in nary:
            return [self._fold(nary[op], w, [A(i) for i in range(len(n.args))])]
        if op in ("bvneg",):
            return [self.mk(I.NEG, w, (A(0),))]
        if op in ("bvnot", "not"):
            return [self.mk(I.NOT, w, (A(0),))]
        if op == "xor":
            return [self.mk(I.XOR, 1, (A(0), A(1)))]
        if op == "=>":
            return [self.mk(I.OR, 1, (self.mk(I.NOT, 1, (A(0),)), A(1)))]
        cmp = {"bvult": (I.ULT, False), "bvule": (I.ULE, False), "bvugt": (I.ULT, True),
               "bvuge": (I.ULE, True), "bvslt": (I.SLT, False), "bvsle": (I.SLE, False),
               "bvsgt": (I.SLT, True), "bvsge": (I.SLE, True), "bvumul_noovfl": (I.UMULNO, False)}
        if op in cmp:
            kop, swap = cmp[op]
            a, b = A(0), A(1)
            if swap:
                a, b = b, a
            return [self.mk(kop, n.args[0].width, (a, b))]
        if op in ("=", "distinct"):
            if any(x.is_array() for x in n.args):
                raise Unsupported("array equality")
            return [self._eq_or_distinct(op, n)]
        if op == "ite":
            if n.is_array():
                raise Unsupported("array-valued ite outside select")
            return [self.mk(I.ITE, w, (A(0), A(1), A(2)))]     # node width (>= both arms)
        if op == "concat":
            word = self._calldata_word(n)
            if word is not None:
                return [word]
            return self.assemble([(self.memo[a.id], a.width) for a in n.args])
        if op == "extract":
            hi, lo = n.params
            src = n.args[0]
            carry = self._carry_pattern(n)
            if carry is not None:
                return [carry]
            return [self.bits(self.memo[src.id], src.width, lo, hi)]
        if op == "zero_extend":
            return [self._narrow(n.args[0])]
        if op == "sign_extend":
            return [self.mk(I.SEXT, w, (A(0),), n.args[0].width)]
        if op == "select":
            return self._select(n.args[0], self.memo[n.args[1].id], n.args[1].width, w)
        if op == "apply":
            fname, dom = n.params
            return self._table(fname, self.memo[n.args[0].id], dom, w, "func")
        raise Unsupported("operator %s" % op)

    def _eq_or_distinct(self, op: str, n: Node) -> LNode:
        args = [self.memo[a.id] for a in n.args]
        w = n.args[0].width

        def eq(x, y):
            parts = [self.mk(I.EQ, self.chunk_width(w, k) if w > CHUNK else w, (x[k], y[k]))
                     for k in range(len(x))]
            return self._fold(I.AND, 1, parts)
        if op == "=":
            return eq(args[0], args[1])
        terms = []
        for i in range(len(args)):
            for j in range(i + 1, len(args)):
                terms.append(self.mk(I.NOT, 1, (eq(args[i], args[j]),)))
        return self._fold(I.AND, 1, terms)

    @staticmethod
    def _is_carry(n: Node) -> bool:
        hi, lo = n.params
        s = n.args[0]
        if hi != lo or s.op != "bvadd" or len(s.args) != 2 or hi != s.width - 1:
            return False
        a, b = s.args
        return (a.op == "zero_extend" and b.op == "zero_extend" and a.params == (1,) and
                b.params == (1,) and a.args[0].width <= CHUNK)

    def _carry_pattern(self, n: Node) -> Optional[LNode]:
        if not self._is_carry(n):
            return None
        x, y = n.args[0].args[0].args[0], n.args[0].args[1].args[0]
        lx, ly = self.lower(x)[0], self.lower(y)[0]
        return self.mk(I.ULT, x.width, (self.mk(I.ADD, x.width, (lx, ly)), lx))

    def _lower_wide(self, n: Node) -> List[LNode]:
        op, w = n.op, n.width
        if op == "bvnum":
            v = n.params[0]
            return [self.const(v >> (CHUNK * k), self.chunk_width(w, k)) for k in range(self.nchunks(w))]
        if op == "var":
            return [self.leaf("%s#%d" % (n.params[0], k), self.chunk_width(w, k), "var",
                              n.params[0], chunk=k) for k in range(self.nchunks(w))]
        if op == "concat":
            return self.assemble([(self.memo[a.id], a.width) for a in n.args])
        if op == "extract":
            src = n.args[0]
            hi, lo = n.params
            return self.assemble([([self.bits(self.memo[src.id], src.width, lo + CHUNK * k,
                                              min(hi, lo + CHUNK * k + CHUNK - 1))],
                                   min(CHUNK, hi - lo + 1 - CHUNK * k))
                                  for k in reversed(range(self.nchunks(w)))])
        if op == "zero_extend":
            src = n.args[0]
            pad = w - src.width
            pieces = []
            while pad > 0:
                pw = min(CHUNK, pad)
                pieces.append(([self.const(0, pw)], pw))
                pad -= pw
            return self.assemble(pieces + [(self.memo[src.id], src.width)])
        if op == "ite":
            c = self._narrow(n.args[0])
            a, b = self.memo[n.args[1].id], self.memo[n.args[2].id]
            return self._ite_chunks(c, a, b)
        if op == "select":
            return self._select(n.args[0], self.memo[n.args[1].id], n.args[1].width, w)
        if op == "apply":
            fname, dom = n.params
            return self._table(fname, self.memo[n.args[0].id], dom, w, "func")
        raise Unsupported("%s on a %d-bit value" % (op, w))

    # -- the calldata word --------------------------------------------------------
    @staticmethod
    def _index_parts(x: Node) -> Tuple[Optional[Node], int]:
        """(base, constant) with x = base + constant (mod 2^256): a numeral
        has no base; ``bvadd`` of a term and a numeral (either order, as LASER
        builds it and as z3's simplify orders it) splits, nested ones too
        (``word(off + 4)`` reads ``(off + 4) + i``); anything else is its own
        base."""
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

    def _calldata_word(self, n: Node) -> Optional[LNode]:
        """LASER's calldata word (``calldata.py:47-54,219-232``)
        ``Concat_{i<32} If(off + i <s size, select(cd, off + i), 0)`` over a
        free array read through its model table (eval form: leaf-keyed
        entries, no constant keys, not argument-keyed) as one chain — the
        ``else`` byte broadcast, one ``CDWE`` per table entry (last entry
        first, so the first match wins) on ``key - off``, then ``CDWX``
        zeroing the bytes past ``size`` — instead of 32 byte lookups, 32
        signed compares, 32 ITEs and 31 CONCATs.  Returns None when ``n`` is
        not that shape.  The byte terms were lowered already (post-order);
        nothing reads them unless another term does."""
        if n.width != 256 or len(n.args) != 32:
            return None
        size = arr = base = None
        c0 = 0
        for i, x in enumerate(n.args):
            if x.op != "ite" or x.width != 8:
                return None
            cond, sel, zero = x.args
            if zero.op != "bvnum" or zero.params[0] != 0 or cond.op != "bvslt" or \
                    sel.op != "select":
                return None
            idx = sel.args[1]
            if cond.args[0] is not idx or idx.width != 256:
                return None
            if i == 0:
                size, arr = cond.args[1], sel.args[0]
                if arr.op != "array":
                    return None
                base, c0 = self._index_parts(idx)
                off = idx
            elif cond.args[1] is not size or sel.args[0] is not arr:
                return None
            else:
                b, c = self._index_parts(idx)
                if b is not base or c != (c0 + i) % (1 << 256):
                    return None
        name = arr.params[0]
        if self.table_ckeys.get(name) or (self.solve and name in self.solve_tables):
            return None
        self.table_kinds[name] = "array"
        entries = self.table_sizes.setdefault(name, self.default_entries)
        o, sz = self._narrow(off), self._narrow(size)
        acc = self.mk(I.BCAST, 256, (self._cell(name, "else", 0, 8)[0],))
        for e in reversed(range(entries)):
            delta = self.mk(I.SUB, 256, (self._cell(name, "key", e, 256)[0], o))
            acc = self.mk(I.CDWE, 256, (acc, delta, self._cell(name, "val", e, 8)[0]))
        return self.mk(I.CDWX, 256, (acc, o, sz))

    def _cell(self, name: str, kind: str, e: int, width: int) -> List[LNode]:
        """The leaves of one model-table cell (key / value / else / constant-
        keyed value), one per 256-bit chunk."""
        tag = {"key": "k%d" % e, "val": "v%d" % e, "else": "else", "cval": "c%d" % e}[kind]
        return [self.leaf("%s#%s#%d" % (name, tag, k), self.chunk_width(width, k), kind,
                          name, chunk=k, entry=e)
                for k in range(self.nchunks(width))]

    # -- arrays and uninterpreted functions ------------------------------------
    def _chunk_eq(self, x: List[LNode], y: List[LNode], w: int) -> LNode:
        parts = [self.mk(I.EQ, self.chunk_width(w, k), (x[k], y[k])) for k in range(len(x))]
        return self._fold(I.AND, 1, parts)

    def _ite_chunks(self, c: LNode, a: List[LNode], b: List[LNode]) -> List[LNode]:
        """Chunk-wise ite.  A chunk's width is the WIDER of its two arms: a
        lowered ``zero_extend`` is its narrow operand itself (values are
        canonical), so one arm may be narrower than the other — taking the
        first arm's width dropped the other arm's high bits (found by the
        full bench-config parity test on C2 DAG 571: a store chain whose
        stored value is a zero-extended 16-bit extract)."""
        return [self.mk(I.ITE, max(x.width, y.width), (c, x, y)) for x, y in zip(a, b)]

    def _table(self, name: str, key: List[LNode], kw: int, vw: int, kind: str) -> List[LNode]:
        """Lookup of a free array / UF in the model's table: first match over
        the constant-keyed entries (``table_ckeys``: the constant indices
        the query reads, keys fixed, one value leaf each), then the
        leaf-keyed entries (key and value leaves), then ``else`` — the
        finite-entries-plus-default interpretation of a z3 model
        (``laser/smt/model.py``).  A lookup at one of the constant keys is
        that entry's value leaf itself."""
        self.table_kinds[name] = kind
        memo_key = (("T", name), tuple(k.id for k in key))
        hit = self.sel_memo.get(memo_key)
        if hit is not None:
            return hit
        entries = self.table_sizes.setdefault(name, self.default_entries)
        ckeys = self.table_ckeys.get(name, [])

        def cell(kind: str, e: int, width: int) -> List[LNode]:
            return self._cell(name, kind, e, width)
        kval = None
        if all(k.op == I.CONST for k in key):
            kval = 0
            for i, k in enumerate(key):
                kval |= k.imm << (CHUNK * i)
        if kval is not None and kval in ckeys:
            acc = cell("cval", ckeys.index(kval), vw)
        elif self.solve and name in self.solve_tables:
            # argument-keyed entries (Ackermann's reduction of a UF / array
            # to one value per distinct argument): lookup j owns entry j,
            # whose KEY is its own argument (computed, reported as a probe)
            # and whose value is a leaf; it reads the first earlier entry
            # with an equal argument, else its own value.  Entries in lookup
            # order with first-match semantics are a consistent model table.
            ents = self.arg_entries.setdefault(name, [])
            val = cell("val", len(ents), vw)
            acc = val
            for k_i, v_i in reversed(ents):
                acc = self._ite_chunks(self._chunk_eq(key, k_i, kw), v_i, acc)
            ents.append((list(key), val))
            self.table_sizes[name] = len(ents)
            if kval is None:
                for i in reversed(range(len(ckeys))):
                    c = [self.const(ckeys[i] >> (CHUNK * k), self.chunk_width(kw, k))
                         for k in range(self.nchunks(kw))]
                    acc = self._ite_chunks(self._chunk_eq(key, c, kw), cell("cval", i, vw), acc)
        else:
            acc = cell("else", 0, vw)
            for e in reversed(range(entries)):
                acc = self._ite_chunks(self._chunk_eq(key, cell("key", e, kw), kw),
                                       cell("val", e, vw), acc)
            if kval is None:         # a symbolic key may equal any constant key
                for i in reversed(range(len(ckeys))):
                    c = [self.const(ckeys[i] >> (CHUNK * k), self.chunk_width(kw, k))
                         for k in range(self.nchunks(kw))]
                    acc = self._ite_chunks(self._chunk_eq(key, c, kw), cell("cval", i, vw), acc)
        self.sel_memo[memo_key] = acc
        return acc

    def _select(self, arr: Node, idx: List[LNode], iw: int, vw: int) -> List[LNode]:
        memo_key = (arr.id, tuple(i.id for i in idx))
        hit = self.sel_memo.get(memo_key)
        if hit is not None:
            return hit
        # walk the store chain iteratively
        chain = []
        a = arr
        while a.op == "store":
            chain.append(a)
            a = a.args[0]
        if a.op == "K":
            base = self.lower(a.args[0])
        elif a.op == "array":
            base = self._table(a.params[0], idx, iw, vw, "array")
        elif a.op == "ite":
            c = self._narrow_node(a.args[0])
            base = self._ite_chunks(c, self._select(a.args[1], idx, iw, vw),
                                    self._select(a.args[2], idx, iw, vw))
        else:
            raise Unsupported("array term %s" % a.op)
        acc = base
        for st in reversed(chain):
            j = self.lower(st.args[1])
            v = self.lower(st.args[2])
            acc = self._ite_chunks(self._chunk_eq(idx, j, iw), v, acc)
        self.sel_memo[memo_key] = acc
        return acc

    def _narrow_node(self, n: Node) -> LNode:
        ch = self.lower(n)
        if len(ch) != 1:
            raise Unsupported("wide condition")
        return ch[0]


# ----------------------------------------------------------------------------
# scheduling + register allocation + emission
# ----------------------------------------------------------------------------

def _schedule(sinks: List[LNode]) -> List[LNode]:
    """Evaluation order: every reachable LNode sorted by (birth, id).

    Source nodes are hash-consed in creation order, and a node is always
    created after its operands, so source-id order is topological; it is also
    the order LASER built the expressions in (``instructions.py`` lowers one
    opcode at a time), which keeps live ranges short.  LNodes born while
    lowering one source node keep their creation order.  A sink (ROOT / OUT)
    is born with its operand, so it is placed right after it and the value
    dies as early as possible."""
    seen = set()
    out = []
    stack = list(sinks)
    while stack:
        n = stack.pop()
        if n.id in seen:
            continue
        seen.add(n.id)
        out.append(n)
        stack.extend(a for a in n.args if a.id not in seen)
    out.sort(key=lambda n: (n.birth, n.id))
    # leaves are born first (the variables exist before the terms over them):
    # each goes right before its first user instead, so it does not hold a
    # register from the start (fewer spills); the translator issues its
    # loads early again where the slot is free (mg_api.cpp, LEAFD)
    lazy: List[LNode] = []
    placed = set()
    for n in out:
        if n.op == I.LEAF:
            continue
        for a in n.args:
            if a.op == I.LEAF and a.id not in placed:
                placed.add(a.id)
                lazy.append(a)
        lazy.append(n)
    lazy += [n for n in out if n.op == I.LEAF and n.id not in placed]
    return lazy


def _schedule_demand(sinks: List[LNode]) -> List[LNode]:
    """Evaluation order driven by the sinks: in sink order, each sink's
    operands not yet scheduled in post-order (a value is computed right
    before the first sink that needs it, not where the source built it)."""
    seen, out = set(), []
    for s in sorted(sinks, key=lambda n: (n.birth, n.id)):
        stack = [(s, False)]
        while stack:
            n, done = stack.pop()
            if done:
                out.append(n)
                continue
            if n.id in seen:
                continue
            seen.add(n.id)
            stack.append((n, True))
            for a in reversed(n.args):
                if a.id not in seen:
                    stack.append((a, False))
    return out


def _alloc_cost(n_lds: int, n_spill: int, n_reload: int, n_ins: int) -> Tuple[int, int, int]:
    """Static cost of an allocation, compared lexicographically: spill slots
    past the LDS tier (per-lane scratch, the HBM round trips a memory-bound
    program waits on), then spill and reload records, then instructions."""
    return (max(0, n_lds - LDS_TIER), n_spill + n_reload, n_ins)


# A/B of the schedule choice (this Python specification only, with
# MYTHRIL_GPU_COMPILER=py: it emits the native compiler's programs, so an
# A/B through it measures the native default against source order)
SCHEDULE_CHOICE = _os.environ.get("MYTHRIL_GPU_SCHEDULE_CHOICE", "1") != "0"
# the sink-driven order is tried only for a program whose source order keeps
# at least this many spill slots in per-lane scratch: the alternated A/B of
# the unconditional choice (profiles/r06/sched2/) gave C3 +3.6 % (source
# order: 15.1 scratch slots per program) but C4 -2.1 % and C5 -0.5 %, whose
# programs mostly keep fewer than 10 (C4 4.4) — there the sink-driven
# order's fewer spill records do not pay for the leaf loads it moves next
# to their readers.  (The env value is for that A/B, Python specification
# only; mg_compile.cpp SCHEDULE_MIN_SCRATCH is the same constant.)
SCHEDULE_MIN_SCRATCH = int(_os.environ.get("MYTHRIL_GPU_SCHEDULE_MIN_SCRATCH", "10"))


def _fuse_roots(order: List[LNode]) -> Tuple[List[LNode], set]:
    """A ROOT that directly follows the instruction computing its operand is
    folded into that instruction (MG_ROOT_FLAG): one dispatch fewer per
    constraint, and the value needs no register if nothing else reads it."""
    out: List[LNode] = []
    fused = set()
    for n in order:
        if n.op == I.ROOT and out and out[-1] is n.args[0] and n.args[0].id not in fused:
            fused.add(n.args[0].id)
            continue
        out.append(n)
    return out, fused


_INPLACE = {I.ADD, I.SUB, I.AND, I.OR, I.XOR, I.NOT, I.NEG, I.ITE, I.CDWE, I.CDWX}


def _allocate(order: List[LNode], const_index: Dict[int, int], fused: set = frozenset(),
              nreg: int = I.NREG, leaf_remat: Optional[str] = None):
    leaf_remat = leaf_remat or LEAF_REMAT
    trash = nreg - 1
    uses: Dict[int, List[int]] = {}
    for i, n in enumerate(order):
        for a in n.args:
            uses.setdefault(a.id, []).append(i)
    ptr: Dict[int, int] = {}
    reg_of: Dict[int, int] = {}
    lds_of: Dict[int, int] = {}
    holder: Dict[int, LNode] = {}          # reg -> value
    # every slot holds values: results nobody reads (fused ROOT conjuncts)
    # are written to a free slot rather than to a dedicated sink slot
    free_regs = list(range(nreg))[::-1]
    reg_clean: Dict[int, bool] = {}        # register's last value had <= 32 bits
    free_lds: List[int] = []
    n_lds = 0
    ins: List[Tuple[int, int, int, int, int, int, int]] = []
    n_spill = n_reload = 0

    def next_use(v: LNode, i: int) -> int:
        u = uses.get(v.id, [])
        p = ptr.get(v.id, 0)
        while p < len(u) and u[p] < i:
            p += 1
        ptr[v.id] = p
        return u[p] if p < len(u) else 1 << 60

    def free_to_drop(v: LNode) -> bool:
        """Evicting v needs no spill: constants are rematerialised, a spilled
        value still has its slot."""
        return v.op == I.CONST or v.id in lds_of

    def droppable_when_full(v: LNode) -> bool:
        """With every spill slot taken a leaf is evicted without a spill
        too: it is regenerated (or reloaded from the input) at its next use —
        more VALU than a reload, so only then."""
        return free_to_drop(v) or v.op == I.LEAF

    def alloc_reg(i: int, protect: set, oldest: bool = False) -> int:
        nonlocal n_lds, n_spill
        if free_regs:
            # reloads take the register free the longest: the translator can
            # then issue them early (mg_api.cpp translate, RELOADD)
            return free_regs.pop(0 if oldest else -1)
        victim, far = None, -1
        for r, v in holder.items():
            if v.id in protect:
                continue
            nu = next_use(v, i)
            if nu > far:
                victim, far = v, nu
        if victim is None:
            raise Unsupported("register pressure")
        if not free_to_drop(victim) and not free_lds and n_lds >= MAX_SPILL:
            # spill slots exhausted: evict the furthest value that needs
            # none (a leaf is regenerated / reloaded from the input instead)
            victim, far = None, -1
            for r, v in holder.items():
                if v.id in protect or not droppable_when_full(v):
                    continue
                nu = next_use(v, i)
                if nu > far:
                    victim, far = v, nu
            if victim is None:
                raise Unsupported("spill budget exceeded")
        r = reg_of.pop(victim.id)
        del holder[r]
        slots_left = bool(free_lds) or n_lds < MAX_SPILL
        if victim.op == I.LEAF and victim.id not in lds_of and leaf_remat != "spill":
            # "scratch": only LDS-tier slots; "scratchK": also the first K
            # scratch slots (a footprint the XCD's L2 still holds)
            tier = LDS_TIER + (int(leaf_remat[7:]) if leaf_remat[7:].isdigit() else 0)
            cheap_free = (free_lds and min(free_lds) < tier) or n_lds < tier
            if leaf_remat == "always" or not cheap_free:
                slots_left = False                       # regenerated at its next use
        if not free_to_drop(victim) and slots_left:
            if free_lds:
                # the lowest free slot: slots below the kernel's LDS tier
                # live in LDS, the rest in per-lane scratch (HBM traffic)
                s = min(free_lds)
                free_lds.remove(s)
            else:
                s = n_lds
                n_lds += 1
            lds_of[victim.id] = s
            ins.append((I.SPILL, 1, trash, r, 0, 0, s))
            n_spill += 1
        return r

    def materialise(v: LNode, r: int):
        nonlocal n_reload
        reg_clean[r] = v.width <= 32
        if v.op == I.CONST:
            ins.append((I.CONST, v.width, r, 0, 0, 0, const_index[v.imm]))
        elif v.id in lds_of:
            ins.append((I.RELOAD, v.width, r, 0, 0, 0, lds_of[v.id]))
            n_reload += 1
        else:                                   # a leaf evicted without a spill
            ins.append((I.LEAF, v.width, r, 0, 0, 0, v.imm))

    def release(v: LNode, i: int):
        if next_use(v, i + 1) >= (1 << 60):
            r = reg_of.pop(v.id, None)
            if r is not None:
                del holder[r]
                free_regs.append(r)
            s = lds_of.pop(v.id, None)
            if s is not None:
                free_lds.append(s)

    for i, n in enumerate(order):
        protect = {a.id for a in n.args}
        for a in n.args:
            if a.id not in reg_of:
                r = alloc_reg(i, protect, oldest=a.op != I.CONST)
                materialise(a, r)
                reg_of[a.id] = r
                holder[r] = a
        slots = [reg_of[a.id] for a in n.args]
        for a in dict.fromkeys(n.args):        # ordered: compiles are reproducible
            release(a, i)
        if n.op in (I.ROOT, I.OUT):
            ins.append((n.op, 1, trash, slots[0], 0, 0, n.imm or 0))
            continue
        flags = I.ROOT_FLAG if n.id in fused else 0
        if not uses.get(n.id):
            if free_regs:
                d = free_regs[-1]            # stays free: the value is dead at once
            else:
                d = alloc_reg(i, set())
                free_regs.append(d)
            # a dead ROOT-fused Bool is not written at all (the translator's NW
            # variants, mg_host.cpp): the register keeps its previous state
            if not (n.id in fused and (n.op in _CMP_OPS or
                                       (n.op in (I.AND, I.OR, I.XOR) and n.width <= 32))):
                reg_clean[d] = n.width <= 32
        else:
            d = None
            # in place: reuse a dying operand's register (the engine then
            # writes the result through the file directly)
            if n.op in _INPLACE and n.width > 32:
                cand = slots[1:3] if n.op == I.ITE else \
                    slots[:1] if n.op in (I.CDWE, I.CDWX) else slots[:2]
                for r in cand:
                    if r in free_regs:
                        free_regs.remove(r)
                        d = r
                        break
            # one-limb results prefer a register whose upper limbs are zero
            if d is None and n.width <= 32:
                for r in reversed(free_regs):
                    if reg_clean.get(r):
                        free_regs.remove(r)
                        d = r
                        break
            # wide results prefer a register whose upper limbs are dirty
            # anyway, keeping the clean ones for one-limb results (their
            # writes then skip the upper limbs: the translator's DC variants)
            if d is None and n.width > 32 and KEEP_CLEAN:
                for r in reversed(free_regs):
                    if not reg_clean.get(r):
                        free_regs.remove(r)
                        d = r
                        break
            if d is None:
                d = alloc_reg(i, set())
            reg_clean[d] = n.width <= 32
            reg_of[n.id] = d
            holder[d] = n
        op = n.op
        a = slots[0] if len(slots) > 0 else 0
        b = slots[1] if len(slots) > 1 else 0
        c = 0
        imm = 0
        width = n.width
        if op == I.CONST:
            imm = const_index[n.imm]
        elif op == I.LEAF:
            imm = n.imm
        elif op in (I.EXTRACT, I.CONCAT, I.SEXT):
            imm = n.imm
        elif op in (I.EQ, I.ULT, I.ULE, I.SLT, I.SLE, I.UMULNO):
            width = n.imm
        elif op == I.ITE:
            c, a, b = slots[0], slots[1], slots[2]
        elif op in (I.CDWE, I.CDWX):
            c = slots[2]
        ins.append((op, width, d, a, b, c, imm, flags))
    return ins, n_lds, n_spill, n_reload


_CMP_OPS = (I.EQ, I.ULT, I.ULE, I.SLT, I.SLE)
# wide results avoid clean registers (a round-2 A/B; the compilers' C ABI
# keeps the flag, mythcc.h keep_clean)
KEEP_CLEAN = True
POOL_CAP = 128          # candidate values per leaf pool


def _pool_values(c: int, w: int) -> List[int]:
    """Candidate values a leaf of width w draws from a constant c it is
    compared with: c itself, c rounded up to a multiple of 64 (keccak UF
    outputs are 64-aligned, keccak_function_manager.py:136-140) and, for
    narrow leaves, every byte-aligned w-bit slice of c (calldata bytes are
    Concat-ed into the words compared with selectors, calldata.py:47-54)."""
    out = [c, (c + 63) & ((1 << 256) - 1) & ~63]
    if w < 256:
        for k in range(0, max(8, c.bit_length()), 8):
            out.append((c >> k) & ((1 << w) - 1))
    return out


def _bits(x: int):
    """Indices of the set bits of x, ascending."""
    while x:
        low = x & -x
        yield low.bit_length() - 1
        x ^= low


def _leaf_pools(order: List[LNode], leaves: List["Leaf"]) -> List[List[int]]:
    """Constraint-guided candidate pools: every comparison (=, <, <=, signed
    or not) makes the constants under it candidates for the leaves under it,
    so a leaf draws the values it is actually tested against instead of any
    constant of the query.  Leaves under no comparison with a constant get
    an empty list (the caller falls back to the whole constant table).
    Leaf and constant sets are bit sets (constants indexed in ascending
    value order, so the POOL_CAP smallest are the lowest bits)."""
    values = sorted({n.imm for n in order if n.op == I.CONST})
    cidx = {v: i for i, v in enumerate(values)}
    under_l: Dict[int, int] = {}
    under_c: Dict[int, int] = {}
    pools: List[Dict[int, None]] = [dict() for _ in leaves]
    done: List[int] = [0] * len(leaves)               # constants already drawn from
    pv: Dict[Tuple[int, int], List[int]] = {}
    M256 = (1 << 256) - 1
    for n in order:                                   # topological
        if n.op == I.LEAF:
            under_l[n.id], under_c[n.id] = 1 << n.imm, 0
            continue
        if n.op == I.CONST:
            under_l[n.id], under_c[n.id] = 0, 1 << cidx[n.imm]
            continue
        ls = cs = 0
        for a in n.args:
            ls |= under_l.get(a.id, 0)
            cs |= under_c.get(a.id, 0)
        if cs.bit_count() > POOL_CAP:                 # keep the walk linear-ish
            keep = 0
            for k, ci in enumerate(_bits(cs)):
                if k == POOL_CAP:
                    break
                keep |= 1 << ci
            cs = keep
        under_l[n.id], under_c[n.id] = ls, cs
        if n.op in _CMP_OPS and cs:
            for li in _bits(ls):
                p = pools[li]
                if len(p) >= POOL_CAP:
                    continue
                new = cs & ~done[li]
                if not new:
                    continue
                done[li] |= new
                w = leaves[li].width
                for ci in _bits(new):
                    c = values[ci]
                    vals = pv.get((c, w))
                    if vals is None:
                        vals = pv[(c, w)] = [v & M256 for v in _pool_values(c, w)]
                    for v in vals:
                        p.setdefault(v)
                        if len(p) >= POOL_CAP:
                            break
                    if len(p) >= POOL_CAP:
                        break
    return [list(p) for p in pools]


CKEY_CAP = 128          # constant-keyed entries per table
CKEY_LINKS = 2048       # symbolic-key lookups x constant keys per table
ARG_ENTRIES_CAP = 64    # solve mode: argument-keyed entries per table (links grow as n^2/2)


def scan_const_keys(nodes: Sequence[Node], cap: int = CKEY_CAP,
                    max_links: int = CKEY_LINKS,
                    sym_counts: Optional[Dict[str, int]] = None) -> Dict[str, List[int]]:
    """The constant indices every free array / UF is read at: ``select`` over
    a store / ite chain ending in a free array, and UF applications, whose
    index is a numeral (calldata bytes at fixed offsets, ``calldata.py:219-
    232``; storage slots at fixed keys, ``account.py:37-62``).  A lookup at a
    symbolic index compares it with every constant key, so a table whose
    symbolic lookups x constant keys exceed ``max_links`` keeps the plain
    leaf-keyed form (e.g. calldata read at a symbolic ABI offset)."""
    out: Dict[str, Dict[int, None]] = {}
    sym: Dict[str, set] = {}

    def bases(a: Node):
        stack, seen = [a], set()
        while stack:
            x = stack.pop()
            if x.id in seen:
                continue
            seen.add(x.id)
            if x.op == "store":
                stack.append(x.args[0])
            elif x.op == "ite":
                stack.extend(x.args[1:])
            elif x.op == "array":
                yield x.params[0]

    def note(name: str, key: Node):
        if key.op == "bvnum":
            d = out.setdefault(name, {})
            if len(d) < cap:
                d.setdefault(key.params[0])
        else:
            sym.setdefault(name, set()).add(key.id)

    for n in topo_order(list(nodes)):
        if n.op == "select":
            for name in bases(n.args[0]):
                note(name, n.args[1])
        elif n.op == "apply":
            note(n.params[0], n.args[0])
    ck = {k: sorted(v) for k, v in out.items() if v and len(sym.get(k, ())) * len(v) <= max_links}
    if sym_counts is not None:
        sym_counts.update({k: len(v) for k, v in sym.items()})
    return ck


def harvest_hints(nodes: Sequence[Node]) -> List[int]:
    """Extra candidate values: every numeral of the query rounded up to a
    multiple of 64 (the keccak UF outputs are constrained to 64-aligned
    intervals, keccak_function_manager.py:136-140) and byte-shifted selector
    constants (calldata words are Concats of bytes)."""
    out = set()
    for n in topo_order(list(nodes)):
        if n.op == "bvnum" and n.width >= 8:
            v = n.params[0]
            out.add((v + 63) & ~63)
            if 0 < v < (1 << 32):
                out.add(v << 224)       # 4-byte selector in the top of a word
    return sorted(out)


def lw_tables(constraints, probes) -> set:
    """Names of every free array / UF the nodes read."""
    out = set()
    for n in topo_order(list(constraints) + list(probes)):
        if n.op == "array":
            out.add(n.params[0])
        elif n.op == "apply":
            out.add(n.params[0])
    return out


# Which compiler compile_constraints runs: "native" (include/mythcc.h, the
# C++ port of this module and solve.py, identical output) or "py" (this
# module; the specification the native one is tested against).
COMPILER = _os.environ.get("MYTHRIL_GPU_COMPILER", "native")


# "auto" (the eval-mode batch path, bench.compile_unit): a program whose
# 256-bit scratch-tier reloads exceed this share of its instructions under
# scratch2 is compiled again under "scratch" (leaves never take a scratch
# slot: regenerated instead).  Round 4, after one-dword narrow spills: C3 /
# C4 run 3.3 / 2.6 % faster under "scratch" (their spills are HBM-bound),
# C2 1.1 % slower (VALU-bound: regeneration costs more than the traffic);
# per program the share is at most 1.8 % on the C2 corpus and a median
# 4.1 / 2.0 / 1.8 % on C3 / C4 / C5 (profiles/r04/remat_r4r/, remat_c2_r4/).
AUTO_SCRATCH_SHARE = 0.02
# ... and a program with (almost) no heavy arithmetic — multiply, division,
# overflow test: the VALU-bound part of C2 — is compiled under "always"
# (leaves never spilled, regenerated at each use: generator v9 and the
# compiled leaf's one-flag path made that cheaper than any spill).  Final
# round-4 kernel, whole workloads (profiles/r04/pol_r4/): "always" C3 / C4 /
# C5 +19 / +19 / +6.6 % over the scratch rule, C2 -2.7 %; every C2 program
# has >= 4 % heavy records, C3 / C4 / C5 programs at most 0.3 %.
AUTO_ALWAYS_HEAVY = 0.01
_HEAVY = (I.MUL, I.UDIV, I.UREM, I.SDIV, I.SREM, I.SMOD, I.UMULNO)


def heavy_share(p: Program) -> float:
    """Multiply / division / overflow-test records per instruction of ``p``."""
    if not len(p.code):
        return 0.0
    op = p.code[:, 0] & 0xFF
    return float(np.isin(op, _HEAVY).sum()) / len(p.code)


def scratch_reload_share(p: Program, lds_tier: int = LDS_TIER) -> float:
    """256-bit reloads from per-lane scratch slots (spill slot index at or
    above the kernel's LDS tier) per instruction of ``p``."""
    code = p.code
    if not len(code):
        return 0.0
    op = code[:, 0] & 0xFF
    width = (code[:, 0] >> 8) & 0x3FF
    hit = (op == I.RELOAD) & (width > 32) & (code[:, 2] >= lds_tier)
    return float(hit.sum()) / len(code)


def compile_constraints(constraints: Sequence[Node], probes: Sequence[Node] = (),
                        table_sizes: Optional[Dict[str, int]] = None,
                        default_entries: int = 2, nreg: int = I.NREG,
                        extra_consts: Sequence[int] = (), leaf_pools: bool = False,
                        const_keys: bool = False, solve: bool = False, search_hints: bool = False,
                        abi_presets: bool = False, leaf_remat: Optional[str] = None) -> Program:
    """Compile constraints (see :func:`compile_constraints_py`) with the
    compiler ``COMPILER`` names, under the leaf policy ``leaf_remat``
    (default ``LEAF_REMAT``; "auto": see ``AUTO_SCRATCH_SHARE`` and
    ``AUTO_ALWAYS_HEAVY``)."""
    global LEAF_REMAT
    policy = leaf_remat or LEAF_REMAT
    if policy == "auto":
        args = (constraints, probes, table_sizes, default_entries, nreg, extra_consts,
                leaf_pools, const_keys, solve, search_hints, abi_presets)
        p = compile_constraints(*args, leaf_remat="scratch2")
        if heavy_share(p) < AUTO_ALWAYS_HEAVY:
            p = compile_constraints(*args, leaf_remat="always")
        elif scratch_reload_share(p) > AUTO_SCRATCH_SHARE:
            p = compile_constraints(*args, leaf_remat="scratch")
        return p
    if COMPILER == "py":
        saved, LEAF_REMAT = LEAF_REMAT, policy
        try:
            return compile_constraints_py(constraints, probes, table_sizes, default_entries, nreg,
                                          extra_consts, leaf_pools, const_keys, solve, search_hints,
                                          abi_presets)
        finally:
            LEAF_REMAT = saved
    from .ccompile import compile_native
    return compile_native(constraints, probes, table_sizes, default_entries, nreg, extra_consts,
                          leaf_pools, const_keys, solve, leaf_remat=policy,
                          search_hints=search_hints, abi_presets=abi_presets)


def compile_constraints_py(constraints: Sequence[Node], probes: Sequence[Node] = (),
                           table_sizes: Optional[Dict[str, int]] = None,
                           default_entries: int = 2, nreg: int = I.NREG,
                           extra_consts: Sequence[int] = (), leaf_pools: bool = False,
                           const_keys: bool = False, solve: bool = False,
                           search_hints: bool = False, abi_presets: bool = False) -> Program:
    """Compile Bool constraint nodes (their conjunction is the root bit) and
    optional probe nodes (256-bit values written per assignment).  ``nreg``
    is the library's register-file size (``Engine.nreg``); ``extra_consts``
    are added to the constant pool (candidate-generator hints).  With
    ``leaf_pools`` every leaf also gets its own candidate pool
    (``_leaf_pools``), stored after the CONST values in the device constant
    table; ``Program.pool_ranges[leaf]`` = (offset, count) in that table.
    With ``const_keys`` every free array / UF gets one constant-keyed entry
    per numeral index it is read at (``scan_const_keys``), so reads at fixed
    offsets are plain leaves instead of lookups in a small leaf-keyed table
    (search mode: every calldata byte a query reads can differ).
    ``solve`` (search mode) builds a program that also constructs part of
    the model instead of guessing it: argument-keyed array / UF entries
    (``_Lowerer._table``) and model construction (``mythril_amd/solve.py``);
    the computed model values come out as probes (``Program.derived`` /
    ``entry_keys``), so such a program is for search, not for evaluating
    caller-supplied assignments.  ``search_hints`` adds the constraints'
    numerals as candidates (:func:`harvest_hints`); ``abi_presets`` pins the
    ABI offset words of calldata read at symbolic offsets (``abi.plan``) and
    compiles the query under them (``Plan.view``, ``Program.presets``)."""
    constraints, probes = list(constraints), list(probes)
    if search_hints:
        extra_consts = list(extra_consts) + harvest_hints(constraints)
    plan = None
    if abi_presets:
        from . import abi
        plan = abi.plan(constraints)
        if plan is not None:
            constraints, probes = plan.view(constraints), plan.view(probes)
    lw = _Lowerer(table_sizes or {}, default_entries)
    lw.solve = solve
    if const_keys or solve:
        sym_counts: Dict[str, int] = {}
        ck = scan_const_keys(list(constraints) + list(probes), sym_counts=sym_counts,
                             cap=256 if solve else CKEY_CAP,
                             max_links=8192 if solve else CKEY_LINKS)
        if const_keys:
            lw.table_ckeys = ck
        # tables read at a bounded number of symbolic keys get argument-keyed
        # entries; the rest keep leaf-keyed ones (calldata at ABI offsets)
        lw.solve_tables = {k for k in lw_tables(constraints, probes)
                           if sym_counts.get(k, 0) <= ARG_ENTRIES_CAP} if solve else set()
    roots: List[LNode] = []
    births: List[int] = []
    for c in constraints:
        if not c.is_bool():
            raise Unsupported("constraint is not Bool")
        roots.append(lw.lower(c)[0])
        births.append(c.id)
    derived_nodes: Dict[int, LNode] = {}
    solver = None
    if solve:
        from .solve import Solver
        solver = Solver(lw)
        roots, derived_nodes = solver.run(roots)
        probe_memo: Dict[int, LNode] = {}
        if solver.dead:                       # a false root: that root alone
            births, probes = births[:1], ()
    sinks: List[LNode] = []
    for r, b in zip(roots, births):
        lw.birth = b
        sinks.append(lw.mk(I.ROOT, 1, (r,), None))
    probe_chunks = 0
    for p in probes:
        if p.is_array():
            raise Unsupported("array probe")
        for ch in lw.lower(p):
            if solver is not None:            # the probe's value under the constructed model
                lw.birth = 0
                ch = solver.rewrite(ch, probe_memo)
            lw.birth = p.id
            sinks.append(lw.mk(I.OUT, 1, (ch,), probe_chunks))
            probe_chunks += 1
    n_user_probes = probe_chunks
    derived: Dict[int, int] = {}
    entry_keys: Dict[str, List[List[int]]] = {}
    if solve:
        def out(n: LNode) -> int:
            nonlocal probe_chunks
            lw.birth = 0                     # right after its operand (short live range)
            sinks.append(lw.mk(I.OUT, 1, (n,), probe_chunks))
            probe_chunks += 1
            return probe_chunks - 1
        for li, e in sorted(derived_nodes.items()):
            derived[li] = out(e)
        memo_e: Dict[int, LNode] = {}
        lw.birth = 0
        for name, ents in (lw.arg_entries.items() if not solver.dead else ()):
            # keys under the constructed model (folded: an ABI offset the
            # model pins makes its reads' keys constants)
            entry_keys[name] = [[out(solver.rewrite(k, memo_e)) for k in key]
                                for key, _ in ents]
    if not sinks:
        sinks.append(lw.mk(I.ROOT, 1, (lw.const(1, 1),), None))
    # comparisons carry their operand width in imm for emission
    for n in list(lw.table.values()):
        if n.op in (I.EQ, I.ULT, I.ULE, I.SLT, I.SLE, I.UMULNO):
            n.imm = n.width
            n.width = 1
    order, fused = _fuse_roots(_schedule(sinks))
    const_values = sorted({n.imm & ((1 << 256) - 1) for n in order if n.op == I.CONST} |
                          {v & ((1 << 256) - 1) for v in extra_consts})
    const_index = {v: i for i, v in enumerate(const_values)}
    ins, n_lds, n_spill, n_reload = _allocate(order, const_index, fused, nreg)
    if not solve and not leaf_pools and SCHEDULE_CHOICE and \
            n_lds - LDS_TIER >= SCHEDULE_MIN_SCRATCH:
        # eval form (round 6): the sink-driven order too, and the one whose
        # allocation costs less (the query streams' calldata words and
        # store-chain reads are built early and read late: C3 -29 % spill
        # records, C4 -48 %; C2's random DAGs mostly keep source order).
        # Search programs keep source order: their compile latency is in
        # front of every query, and their leaf pools follow that order.
        order2, fused2 = _fuse_roots(_schedule_demand(sinks))
        try:
            alt = _allocate(order2, const_index, fused2, nreg)
        except Unsupported:
            alt = None
        if alt is not None and _alloc_cost(alt[1], alt[2], alt[3], len(alt[0])) < \
                _alloc_cost(n_lds, n_spill, n_reload, len(ins)):
            ins, n_lds, n_spill, n_reload = alt
            order, fused = order2, fused2
    code = np.zeros((len(ins), 4), dtype=np.uint32)
    for k, (op, width, d, a, b, c, imm, *fl) in enumerate(ins):
        code[k, 0] = op | (width << 8) | (fl[0] if fl else 0)
        code[k, 1] = I.w1(d, a, b, c)
        code[k, 2] = imm
    table = list(const_values)
    pool_ranges: List[Tuple[int, int]] = []
    if leaf_pools:
        for li, p in enumerate(_leaf_pools(order, lw.leaves)):
            if p:
                pool_ranges.append((len(table), len(p)))
                table.extend(p)
            else:
                pool_ranges.append((0, len(const_values)))
    consts = np.frombuffer(b"".join(v.to_bytes(32, "little") for v in table),
                           dtype="<u4").reshape(-1, 8).astype(np.uint32)
    hist: Dict[str, int] = {}
    for n in order:
        hist[I.OPNAME[n.op]] = hist.get(I.OPNAME[n.op], 0) + 1
    stats = {"lnodes": len(order), "n_ins": len(ins), "spills": n_spill, "reloads": n_reload,
             "hist": hist}
    ckeys = {k: v for k, v in lw.table_ckeys.items() if k in lw.table_kinds}
    tsizes = dict(lw.table_sizes)
    for name in lw.solve_tables & set(lw.table_kinds):
        # no leaf-keyed entries: the model's entries are the argument-keyed ones
        tsizes[name] = len(lw.arg_entries.get(name, ()))
    prog = Program(code, consts, const_values, lw.leaves, n_lds, probe_chunks,
                   len(constraints), tsizes, lw.table_kinds, ckeys, stats, pool_ranges,
                   derived, entry_keys, n_user_probes)
    prog.nreg = nreg
    if plan is not None:
        prog.presets = plan
    return prog
