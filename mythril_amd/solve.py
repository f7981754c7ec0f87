"""Search-mode model construction (``compile_constraints(..., solve=True)``).

The witness search guesses a model per candidate; a guess that must hit one
value out of 2^256 (``calldata[0..3] = selector``, ``sender in ACTORS``,
``keccak(x) = H``) never lands.  This pass turns such constraints into
*definitions*: a leaf whose value a conjunct pins is computed from the
other leaves instead of guessed, and every use of the leaf reads the
computed value.  The program still evaluates every ORIGINAL constraint on
the constructed model — a definition can only make a candidate more likely
to satisfy the query, never accept a wrong one — and reports each defined
leaf's value as a probe (``Program.derived``), so witnesses are ordinary
models (``assign.unpack``).

Steps, over the lowered DAG (``ir._Lowerer``):

* **folding** (``_fold``): constant ``=`` / ``ite`` conditions / Boolean
  ``and or not`` with constant operands, ``ite(c, x, x)``, ``not not x``;
* **atoms** (``_atoms``): each root is split into conjuncts through ``and``,
  De Morgan over ``not or``, and equalities with a constant are pushed
  through bit-field structure — ``concat`` (per part), ``extract`` (of a
  concat / extract / ite), ``and`` with a low mask, ``ite`` with a
  constant arm (``ite(c, k1, k2) = k1`` is ``c``; ``ite(c, x, k2) = k`` is
  ``c and x = k`` when ``k2 != k``, otherwise ``x = k`` suffices);
* **definitions** (``_define``): an atom ``leaf = e`` (``e`` not depending on
  the leaf, definitions followed transitively) defines the leaf as ``e``;
  ``ite(c, leaf, y) = e`` defines the leaf as ``e`` (sufficient); an atom
  ``leaf = k1 or ... or leaf = kn`` (a domain: ``sender in ACTORS``)
  defines the leaf as one of the ``k_i`` picked by a fresh 8-bit selector
  leaf (kind ``aux``: generated, not part of the model);
* up to ``PASSES`` rounds, since a definition can fold later conjuncts into
  new atoms (``calldata[i] = b`` makes the ``ite(i < calldatasize, ...)``
  guards of other reads constant).

Mythril's own solver never sees these programs; this is the GPU search's
way of reaching the models z3 would construct for the same queries
(``laser/ethereum/keccak_function_manager.py``'s
``inverse(f(x)) = x``, ``transaction/symbolic.py``'s actor ``Or``, the
dispatcher's selector equalities)."""

from __future__ import annotations

from typing import Dict, List, Optional

from . import irdefs as I

PASSES = 6
MAX_DOMAIN = 16          # constants in an ``or`` of equalities made a domain
MAX_BRANCHES = 4         # disjuncts of an ``or`` split by a selector
MAX_OR = 64              # such splits per program
BRANCH_DEPTH = 2
SELECTOR_WIDTH = 8
MAX_REFUSALS = 4         # definitions refused after killing a root, per run


_PREDICATES = (I.EQ, I.ULT, I.ULE, I.SLT, I.SLE, I.UMULNO)


def _bit_indices(x: int):
    while x:
        low = x & -x
        yield low.bit_length() - 1
        x ^= low


class _Overlay(dict):
    """A rewrite memo layered over another: reads fall through to the
    parent, writes stay local.  ``_branches`` tries each disjunct's
    definitions on top of the run's memo (valid for the definitions in force
    before the disjunct: rewrite re-folds the entries a new definition
    reaches) and drops the layer when the definitions are rolled back."""
    __slots__ = ("parent",)

    def __init__(self, parent):
        super().__init__()
        self.parent = parent

    def get(self, k, d=None):
        v = dict.get(self, k)
        return self.parent.get(k, d) if v is None else v

    def __getitem__(self, k):
        v = dict.get(self, k)
        return self.parent[k] if v is None else v


def _is_false(x) -> bool:
    return x.op == I.CONST and not x.imm & 1


def _mask(w: int) -> int:
    return (1 << w) - 1


class Solver:
    def __init__(self, lw):
        self.lw = lw
        self.repl: Dict[int, "object"] = {}          # LEAF LNode id -> definition
        self.one = lw.const(1, 1)
        self.zero = lw.const(0, 1)
        self.n_aux = 0
        self.n_branch = 0
        self.selectors: set = set()              # LEAF ids of branch / domain selectors
        self.or_seen: set = set()                # ``or`` atoms already split
        self.dep: Dict[int, int] = {}            # LNode id -> leaf bit set
        self.ivl: Dict[int, tuple] = {}          # LNode id -> unsigned interval
        self.joint_done: set = set()             # expressions whose bounds were joined
        self.clean: set = set()                  # ids of rewrite results
        self.leaf_imm: Dict[int, int] = {}       # defined LEAF id -> leaf index
        self.leaf_node: Dict[int, object] = {}   # defined LEAF id -> the LEAF node
        self._dm = None                          # bit set of the defined leaves
        self._memo: Dict[int, object] = {}       # the run's rewrite memo (run)
        # LEAF id -> generation of a branch's stand-in for an undefined value
        # (a stand-in may be split again by a later ``or``, to BRANCH_DEPTH)
        self.depth: Dict[int, int] = {}
        self.unsat = False
        self.dead = False                        # run: a root folded to false
        self.refused: set = set()                # leaves (_key) whose definition killed a root
        # a generated leaf's ordinal in this construction (run repeats the
        # construction; the same ordinal is the same choice)
        self.aux_seq: Dict[int, int] = {}
        # leaves defined from an overflow test's atoms (the module's check)
        self._wrap_ctx = False
        self.wrap_defs: set = set()

    # -- rewriting -------------------------------------------------------------
    def _interval(self, n):
        """Unsigned [lo, hi] of a value (canonical: a node of width w is
        below 2^w); exact for constants, sums that cannot wrap, ite."""
        r = self.ivl.get(n.id)
        if r is not None:
            return r
        top = _mask(n.width)
        if n.op == I.CONST:
            r = (n.imm, n.imm)
        elif n.op == I.ADD:
            (la, ha), (lb, hb) = self._interval(n.args[0]), self._interval(n.args[1])
            r = (la + lb, ha + hb) if ha + hb <= top else (0, top)
        elif n.op == I.ITE:
            (la, ha), (lb, hb) = self._interval(n.args[1]), self._interval(n.args[2])
            r = (min(la, lb), max(ha, hb))
        elif n.op in _PREDICATES:
            r = (0, 1)
        else:
            r = (0, top)
        self.ivl[n.id] = r
        return r

    def _cmp_fold(self, op, w, a, b):
        """ULT / ULE / SLT / SLE decided by the operands' intervals, or None."""
        (la, ha), (lb, hb) = self._interval(a), self._interval(b)
        if op in (I.SLT, I.SLE):
            half = 1 << (w - 1)
            if ha >= half or hb >= half:
                return None                      # not both non-negative
        if op in (I.ULT, I.SLT):
            if ha < lb:
                return self.one
            if la >= hb:
                return self.zero
        else:
            if ha <= lb:
                return self.one
            if la > hb:
                return self.zero
        return None

    def _const_fold(self, x, args):
        """Bit-vector ops over constants."""
        w, op = x.width, x.op
        v = [a.imm for a in args]
        m = _mask(w)
        if op == I.CONCAT:
            return (v[0] << x.imm | v[1]) & m
        if op == I.EXTRACT:
            return (v[0] >> x.imm) & m
        if op == I.AND:
            return v[0] & v[1] & m
        if op == I.OR:
            return (v[0] | v[1]) & m
        if op == I.XOR:
            return (v[0] ^ v[1]) & m
        if op == I.SUB:
            return (v[0] - v[1]) & m
        if op == I.MUL:
            return (v[0] * v[1]) & m
        if op == I.NOT:
            return ~v[0] & m
        return None

    def _fold(self, x, args):
        lw, op = self.lw, x.op
        if op in (I.CONCAT, I.EXTRACT, I.AND, I.OR, I.XOR, I.SUB, I.MUL, I.NOT) and \
                all(a.op == I.CONST for a in args):
            c = self._const_fold(x, args)
            if c is not None:
                return lw.const(c, x.width)
        if op in (I.ULT, I.ULE, I.SLT, I.SLE) and not all(a.op == I.CONST for a in args):
            r = self._cmp_fold(op, x.width, args[0], args[1])
            if r is not None:
                return r
        if op == I.EQ:
            a, b = args
            if a is b:
                return self.one
            if a.op == I.CONST and b.op == I.CONST:
                return self.one if a.imm == b.imm else self.zero
            # y + c1 = y + c2 (and y + c = y): symbolic ABI offsets that differ
            # by a constant never alias
            ya, ca = (a.args[0], a.args[1].imm) if a.op == I.ADD and a.args[1].op == I.CONST \
                else (a, 0)
            yb, cb = (b.args[0], b.args[1].imm) if b.op == I.ADD and b.args[1].op == I.CONST \
                else (b, 0)
            if ya is yb and a.width == b.width and ya.op != I.CONST:
                return self.one if ca == cb else self.zero
            (la, ha), (lb, hb) = self._interval(a), self._interval(b)
            if ha < lb or hb < la:                   # disjoint ranges (a keccak
                return self.zero                     # interval vs a small slot)
        elif op == I.ADD:
            a, b = args
            if a.op == I.CONST and b.op != I.CONST:
                a, b = b, a
            if b.op == I.CONST:
                w = x.width
                if a.op == I.CONST:
                    return lw.const((a.imm + b.imm) & _mask(w), w)
                if b.imm == 0 and a.width <= w:
                    return a
                if a.op == I.ADD and a.width == w and a.args[1].op == I.CONST:
                    # (y + c1) + c2 = y + (c1 + c2): ABI offsets off + 4 + i
                    return lw.mk(I.ADD, w, (a.args[0], lw.const((a.args[1].imm + b.imm) & _mask(w), w)))
                if (a, b) != args:
                    return lw.mk(I.ADD, w, (a, b))
        elif op in (I.ULT, I.ULE, I.SLT, I.SLE) and all(a.op == I.CONST for a in args):
            a, b = args[0].imm, args[1].imm
            if op in (I.SLT, I.SLE):
                half = 1 << (x.width - 1)
                a, b = a - 2 * half if a >= half else a, b - 2 * half if b >= half else b
            return self.one if (a < b if op in (I.ULT, I.SLT) else a <= b) else self.zero
        elif op == I.ITE:
            c = args[0]
            if c.op == I.CONST:
                return args[1] if c.imm & 1 else args[2]
            if args[1] is args[2]:
                return args[1]
        elif op in (I.AND, I.OR) and x.width == 1:
            absorb = 0 if op == I.AND else 1
            rest = []
            for a in args:
                if a.op == I.CONST:
                    if (a.imm & 1) == absorb:
                        return a if a.width == 1 else lw.const(absorb, 1)
                    continue
                rest.append(a)
            if not rest:
                return lw.const(1 - absorb, 1)
            if len(rest) == 1:
                return rest[0]
            if rest[0] is rest[1]:
                return rest[0]
        elif op == I.NOT and x.width == 1:
            a = args[0]
            if a.op == I.CONST:
                return lw.const(1 - (a.imm & 1), 1)
            if a.op == I.NOT and a.width == 1:
                return a.args[0]
        if all(a is b for a, b in zip(args, x.args)):
            return x
        return lw.mk(op, x.width, args, x.imm)

    def _dep(self, n) -> int:
        """Bit set (by leaf index) of the leaves under ``n``."""
        dep = self.dep
        d = dep.get(n.id)
        if d is not None:
            return d
        stack = [n]
        while stack:
            x = stack[-1]
            if x.id in dep:
                stack.pop()
                continue
            pend = [a for a in x.args if a.id not in dep]
            if pend:
                stack.extend(pend)
                continue
            stack.pop()
            if x.op == I.LEAF:
                v = 1 << x.imm
            else:
                v = 0
                for a in x.args:
                    v |= dep[a.id]
            dep[x.id] = v
        return dep[n.id]

    def _defmask(self) -> int:
        if self._dm is None:
            m = 0
            for k in self.repl:
                m |= 1 << self.leaf_imm[k]
            self._dm = m
        return self._dm

    def rewrite(self, n, memo: Dict[int, object]):
        """``n`` with every defined leaf replaced by its definition (followed
        transitively) and folded.  A node that is already a rewrite result
        (``clean``: folding cannot change it) over undefined leaves only is
        its own result — the walk does not enter it.

        ``memo`` may outlive definitions: an entry stays valid while no leaf
        of its result has been defined since (results hold undefined leaves
        only), so a pass re-folds just the nodes a new definition reaches."""
        dm = self._defmask()
        clean, dep, get = self.clean, self._dep, memo.get
        stack = [(n, False)]
        while stack:
            x, done = stack.pop()
            if not done:
                r = get(x.id)
                if r is not None and not dep(r) & dm:
                    continue
            if x.op == I.LEAF:
                e = self.repl.get(x.id)
                if e is None:
                    memo[x.id] = x
                    continue
                r = get(e.id)
                if r is not None and not dep(r) & dm:
                    memo[x.id] = r
                else:
                    stack.append((x, False))
                    stack.append((e, False))
                continue
            if not x.args:
                memo[x.id] = x
                continue
            if not done:
                if x.id in clean and not dep(x) & dm:
                    memo[x.id] = x
                    continue
                stack.append((x, True))
                for a in x.args:
                    r = get(a.id)
                    if r is None or dep(r) & dm:
                        stack.append((a, False))
                continue
            r = self._fold(x, tuple(memo[a.id] for a in x.args))
            clean.add(r.id)
            memo[x.id] = r
        return memo[n.id]

    # -- small constructors ------------------------------------------------------
    def _not(self, a):
        if a.op == I.CONST:
            return self.lw.const(1 - (a.imm & 1), 1)
        if a.op == I.NOT and a.width == 1:
            return a.args[0]
        return self.lw.mk(I.NOT, 1, (a,))

    def _eq(self, a, k: int):
        if k >> a.width:
            return self.zero
        if a.op == I.CONST:
            return self.one if a.imm == k else self.zero
        return self.lw.mk(I.EQ, a.width, (a, self.lw.const(k, a.width)))

    def _ext(self, a, off: int, k: int):
        if off == 0 and k == a.width:
            return a
        if a.op == I.CONST:
            return self.lw.const((a.imm >> off) & _mask(k), k)
        if a.op == I.EXTRACT:
            return self._ext(a.args[0], a.imm + off, k)
        return self.lw.mk(I.EXTRACT, k, (a,), off)

    @staticmethod
    def _concat_parts(a):
        """(high part, low part, low width) of a CONCAT (the 256-bit funnel
        form keeps a full-width high operand: only its low bits count)."""
        hi, lo = a.args
        lw_ = a.imm
        return hi, lw_, lo

    def _hi(self, a):
        hi, lw_, _ = self._concat_parts(a)
        hw = a.width - lw_
        return hi if hi.width == hw else self._ext(hi, 0, hw)

    # -- atoms -----------------------------------------------------------------
    def _split_eq(self, x) -> Optional[list]:
        """Conjuncts equivalent to (or sufficient for) ``x = k`` pushed through
        the structure of ``x``; None when nothing applies."""
        a, b = x.args
        if a.op == I.CONST and b.op != I.CONST:
            a, b = b, a
        if b.op != I.CONST:
            return None
        k = b.imm
        if a.op in _PREDICATES or (a.op in (I.AND, I.OR, I.NOT) and a.width == 1):
            if k > 1:
                return [self.zero]
            return [a] if k else [self._not(a)]
        if a.op == I.ITE:
            c, p, q = a.args
            if p.op == I.CONST and q.op == I.CONST:
                if p.imm == k and q.imm == k:
                    return []
                if p.imm == k:
                    return [c]
                if q.imm == k:
                    return [self._not(c)]
                return [self.zero]
            if q.op == I.CONST:
                if q.imm != k:
                    return [c, self._eq(p, k)]
                # q = k: p = k suffices — unless p can never be k (its range
                # excludes it), then c must be false
                lo, hi = self._interval(p)
                return [self._eq(p, k)] if lo <= k <= hi else [self._not(c)]
            if p.op == I.CONST:
                if p.imm != k:
                    return [self._not(c), self._eq(q, k)]
                # p = k (a first-match table read ite(x = k0, h0, v) = h0):
                # v = k suffices — unless v can never be k, then x = k0
                lo, hi = self._interval(q)
                return [self._eq(q, k)] if lo <= k <= hi else [c]
            return [self._eq(p, k), self._eq(q, k)]             # sufficient
        if a.op == I.AND and a.width > 1:
            m, z = a.args
            if z.op == I.CONST:
                m, z = z, m
            if m.op != I.CONST:
                return None
            if k & ~m.imm:
                return [self.zero]
            if m.imm & _mask(z.width) == _mask(z.width):
                return [self._eq(z, k)]
            low = m.imm & _mask(z.width)
            if low & (low + 1) == 0:                              # a low mask 2^j - 1
                return [self._eq(self._ext(z, 0, low.bit_length()), k)]
            return None
        if a.op == I.CONCAT:
            if k >> a.width:
                return [self.zero]
            _, lw_, lo = self._concat_parts(a)
            return [self._eq(lo, k & _mask(lw_)), self._eq(self._hi(a), k >> lw_)]
        if a.op == I.EXTRACT:
            y, off, w = a.args[0], a.imm, a.width
            if y.op == I.CONCAT:
                _, lw_, lo = self._concat_parts(y)
                if off + w <= lw_:
                    return [self._eq(self._ext(lo, off, w), k)]
                hi = self._hi(y)
                if off >= lw_:
                    return [self._eq(self._ext(hi, off - lw_, w), k)]
                n_lo = lw_ - off
                return [self._eq(self._ext(lo, off, n_lo), k & _mask(n_lo)),
                        self._eq(self._ext(hi, 0, w - n_lo), k >> n_lo)]
            if y.op == I.ITE:
                c, p, q = y.args
                return [self.lw.mk(I.EQ, w, (self.lw.mk(I.ITE, w, (c, self._ext(p, off, w),
                                                                    self._ext(q, off, w))),
                                             self.lw.const(k, w)))]
        return None

    def _neg_eq(self, y):
        """``not (ite(c, k1, k2) = k)`` as a condition on ``c``."""
        a, b = y.args
        if a.op == I.CONST and b.op != I.CONST:
            a, b = b, a
        if b.op != I.CONST:
            return None
        if a.op in _PREDICATES or (a.op in (I.AND, I.OR, I.NOT) and a.width == 1):
            return self.one if b.imm > 1 else (a if b.imm == 0 else self._not(a))
        if a.op != I.ITE:
            return None
        c, p, q = a.args
        if p.op != I.CONST or q.op != I.CONST:
            return None
        k = b.imm
        if p.imm == k and q.imm == k:
            return self.zero
        if p.imm == k:
            return self._not(c)
        if q.imm == k:
            return c
        return self.one

    def _atoms(self, root, memo) -> list:
        out, stack = [], [self.rewrite(root, memo)]
        seen = set()
        while stack:
            x = stack.pop()
            if x.id in seen:
                continue
            seen.add(x.id)
            if x.op == I.CONST:
                if not x.imm & 1:
                    self.unsat = True
                continue
            if x.op == I.AND and x.width == 1:
                stack.extend(x.args)
                continue
            if x.op == I.NOT and x.width == 1:
                y = x.args[0]
                if y.op == I.OR and y.width == 1:
                    stack.extend(self._not(a) for a in y.args)
                    continue
                if y.op == I.EQ:
                    r = self._neg_eq(y)
                    if r is not None:
                        stack.append(r)
                        continue
                if y.op in (I.ULT, I.ULE, I.SLT, I.SLE):
                    pass                         # a negated bound: handled below
                else:
                    out.append(x)
                if y.op not in (I.ULT, I.ULE, I.SLT, I.SLE) and y.op == I.UMULNO and \
                        y.args[1].op != I.CONST:
                    # a * b >= 2^w (BVMulNoOverflow negated): b = 2^w - 1
                    # overflows for every a > 1, b = 2^(w-1) for every even a
                    # with a zero product (what a later balance check needs:
                    # BECToken's batchTransfer) — a split between the two
                    b_ = y.args[1]
                    w_ = y.width
                    stack.append(self.rewrite(self.lw.mk(I.OR, 1, (
                        self._eq(b_, _mask(b_.width)), self._eq(b_, 1 << (w_ - 1)))), memo))
                if y.op not in (I.ULT, I.ULE, I.SLT, I.SLE):
                    continue
            if x.op == I.EQ:
                parts = self._split_eq(x)
                if parts is not None:
                    stack.extend(self.rewrite(p, memo) for p in parts)
                    continue
            if x.op == I.ULT and x.args[0].op == I.ADD and x.args[1] in x.args[0].args:
                # a + b < a (the carry BVAddNoOverflow tests): b = 2^w - 1
                # overflows for every a > 0 (a sufficient condition)
                s_, a_ = x.args[0], x.args[1]
                other = s_.args[1] if s_.args[0] is a_ else s_.args[0]
                out.append(x)
                if other.op != I.CONST:
                    stack.append(self.rewrite(self._eq(other, _mask(other.width)), memo))
                continue
            if x.op == I.OR and x.width == 1:
                le = self._as_ule(x)
                if le is not None:
                    stack.append(le)
                    continue
            b = self._bound(x)
            if b is not None and b[0].op in (I.ITE, I.CONCAT, I.MUL):
                parts = self._split_bound(*b)
                if parts is not None:
                    if b[0].op != I.ITE:
                        out.append(x)            # (a sufficient condition only)
                    stack.extend(self.rewrite(p, memo) for p in parts)
                    continue
            if b is None:
                parts = self._order_via_arm(x)
                if parts is not None:
                    out.append(x)
                    stack.extend(self.rewrite(p, memo) for p in parts)
                    continue
            out.append(x)
        return out

    def _order_via_arm(self, x) -> Optional[list]:
        """``a <= s`` / ``a < s`` with ``s`` an ite tree of constants (a
        storage read: known values, else 0): commit to the path that gives
        ``s`` its largest value and bound ``a`` by it (sufficient)."""
        neg = x.op == I.NOT and x.width == 1
        y = x.args[0] if neg else x
        if y.op not in (I.ULT, I.ULE):
            return None
        a, s = y.args
        strict = y.op == I.ULT
        if neg:                                    # not (s' < a') = a' <= s'
            a, s, strict = s, a, not strict
        if s.op != I.ITE:
            return None
        best = self._max_arm(s)
        if best is None:
            return None
        k, conds = best
        hi = k - 1 if strict else k
        if hi < 0:
            return None
        return conds + self._mk_bound(a, 0, hi, y.width)

    def _max_arm(self, s, depth: int = 8):
        """(largest constant an ite tree can select, the conditions that
        select it) over constant arms only."""
        best = None
        stack = [(s, [], 0)]
        while stack:
            n, conds, d = stack.pop()
            if n.op == I.CONST:
                if best is None or n.imm > best[0]:
                    best = (n.imm, conds)
            elif n.op == I.ITE and d < depth:
                c = n.args[0]
                stack.append((n.args[1], conds + [c], d + 1))
                stack.append((n.args[2], conds + [self._not(c)], d + 1))
        return best

    def _as_ule(self, x):
        """``a < b or a = b`` (how LASER writes ``ULE`` / ``UGE``) as one
        ``a <= b``."""
        p, q = x.args
        for lt, eq in ((p, q), (q, p)):
            if lt.op == I.ULT and eq.op == I.EQ and \
                    {eq.args[0].id, eq.args[1].id} == {lt.args[0].id, lt.args[1].id}:
                return self.lw.mk(I.ULE, lt.width, lt.args)
        return None

    # -- bounds ------------------------------------------------------------------
    @staticmethod
    def _bound(x):
        """``x`` as ``lo <= e <= hi`` (unsigned, inclusive) with constant
        bounds: (e, lo, hi, operand width), or None.  A signed comparison
        with a non-negative constant gives the non-negative half (exact for
        ``k < e``, sufficient for ``e < k``: the calldata guards
        ``offset < calldatasize``)."""
        neg = False
        if x.op == I.NOT and x.width == 1:
            x, neg = x.args[0], True
        if x.op not in (I.ULT, I.ULE, I.SLT, I.SLE):
            return None
        a, b = x.args
        w = x.width
        top = _mask(w)
        strict = x.op in (I.ULT, I.SLT)
        if x.op in (I.SLT, I.SLE):
            if neg:
                return None
            top = _mask(w - 1)
            k = b.imm if b.op == I.CONST else (a.imm if a.op == I.CONST else None)
            if k is None or k > top or (a.op == I.CONST) == (b.op == I.CONST):
                return None
        if b.op == I.CONST and a.op != I.CONST:
            k = b.imm
            # a < k | a <= k ; negated: a >= k | a > k
            if not neg:
                return (a, 0, k - 1 if strict else k, w) if (k or not strict) else None
            return (a, k if strict else k + 1, top, w) if (k < top or strict) else None
        if a.op == I.CONST and b.op != I.CONST:
            k = a.imm
            # k < b | k <= b ; negated: b <= k | b < k
            if not neg:
                return (b, k + 1 if strict else k, top, w) if (k < top or not strict) else None
            return (b, 0, k if strict else k - 1, w) if (k or strict) else None
        return None

    def _mk_bound(self, e, lo: int, hi: int, w: int) -> list:
        out = []
        if lo > hi:
            return [self.zero]
        if lo > 0:
            out.append(self.lw.mk(I.ULE, w, (self.lw.const(lo, w), e)))
        if hi < _mask(w):
            out.append(self.lw.mk(I.ULE, w, (e, self.lw.const(hi, w))))
        return out

    def _split_ite_bound(self, e, lo, hi, w) -> Optional[list]:
        """``lo <= ite(c, k, y) <= hi``: ``y`` in range suffices when ``k`` is
        (else ``not c`` is needed too)."""
        c, p, q = e.args
        if p.op == I.CONST and q.op != I.CONST:
            inside = lo <= p.imm <= hi
            return self._mk_bound(q, lo, hi, w) + ([] if inside else [self._not(c)])
        if q.op == I.CONST and p.op != I.CONST:
            inside = lo <= q.imm <= hi
            return self._mk_bound(p, lo, hi, w) + ([] if inside else [c])
        if p.op != I.CONST and q.op != I.CONST:
            return self._mk_bound(p, lo, hi, w) + self._mk_bound(q, lo, hi, w)   # sufficient
        return None

    def _split_bound(self, e, lo, hi, w) -> Optional[list]:
        if e.op == I.ITE:
            return self._split_ite_bound(e, lo, hi, w)
        if e.op == I.CONCAT:
            # x = h . l in [lo, hi] with hi < 2^|l|: h = 0 and l in [lo, hi]
            # (exact, down the concat chain); a larger hi: h < hi >> |l|
            # (any l; sufficient)
            out = []
            while e.op == I.CONCAT:
                _, lw_, l_ = self._concat_parts(e)
                if hi >> lw_:
                    break
                out.append(self._eq(self._hi(e), 0))
                e = l_
            if e.op != I.CONCAT:
                return out + self._mk_bound(e, lo, hi, e.width)
            if lo:
                return out or None
            _, lw_, _ = self._concat_parts(e)
            h = self._hi(e)
            return out + self._mk_bound(h, 0, (hi >> lw_) - 1, h.width)
        if lo:
            return None
        if e.op == I.MUL:
            # a * b <= hi: both factors below 2^(k/2) with 2^k <= hi + 1
            k = (hi + 1).bit_length() - 1
            a, b = e.args
            return (self._mk_bound(a, 0, (1 << (k // 2)) - 1, w) +
                    self._mk_bound(b, 0, (1 << (k - k // 2)) - 1, w))
        return None

    # -- definitions -------------------------------------------------------------
    def _depends(self, e, leaf) -> bool:
        seen, stack = set(), [e]
        while stack:
            x = stack.pop()
            if x is leaf:
                return True
            if x.id in seen:
                continue
            seen.add(x.id)
            if x.op == I.LEAF:
                d = self.repl.get(x.id)
                if d is not None:
                    stack.append(d)
                continue
            stack.extend(x.args)
        return False

    def _try_define(self, leaf, e) -> bool:
        if leaf.op != I.LEAF or leaf.id in self.repl:
            return False
        if leaf.id in self.selectors and e.op != I.CONST:
            return False                         # a selector only commits to a branch
        if self.refused and self._key(leaf.id) in self.refused:
            return False                         # its definition killed a root (run)
        if e.width > leaf.width and not (e.op == I.CONST and e.imm >> leaf.width == 0):
            return False
        if self._depends(e, leaf):
            return False
        self.repl[leaf.id] = e
        if self._wrap_ctx:
            self.wrap_defs.add(leaf.id)
        self.leaf_imm[leaf.id] = leaf.imm
        self.leaf_node[leaf.id] = leaf
        self._dm = None
        return True

    @staticmethod
    def _ite_leaves(x, limit: int = 16) -> list:
        """Leaves an ite tree (through its arms, not its conditions) can
        select, innermost-else last."""
        out, stack = [], [x] if x.op == I.ITE else []
        while stack and len(out) < limit:
            y = stack.pop()
            for arm in (y.args[1], y.args[2]):
                if arm.op == I.LEAF:
                    out.append(arm)
                elif arm.op == I.ITE:
                    stack.append(arm)
        return out

    def _domain(self, x) -> bool:
        """``leaf = k1 or ... or leaf = kn``: the leaf becomes a selector-picked
        constant."""
        disj, stack = [], [x]
        while stack:
            y = stack.pop()
            if y.op == I.OR and y.width == 1:
                stack.extend(y.args)
            else:
                disj.append(y)
        if len(disj) > MAX_DOMAIN:
            return False
        leaf, ks = None, []
        for d in disj:
            if d.op != I.EQ:
                return False
            a, b = d.args
            if a.op == I.CONST:
                a, b = b, a
            if a.op != I.LEAF or b.op != I.CONST or (leaf is not None and a is not leaf):
                return False
            leaf = a
            if b.imm not in ks:
                ks.append(b.imm)
        if leaf is None or leaf.id in self.repl:
            return False
        lw = self.lw
        sel = self._selector()
        span = 1 << SELECTOR_WIDTH
        e = lw.const(ks[-1], leaf.width)
        for i in reversed(range(len(ks) - 1)):
            t = lw.const(span * (i + 1) // len(ks), SELECTOR_WIDTH)
            e = lw.mk(I.ITE, leaf.width, (lw.mk(I.ULT, SELECTOR_WIDTH, (sel, t)),
                                          lw.const(ks[i], leaf.width), e))
        return self._try_define(leaf, e)

    def _selector(self):
        sel = self._aux(SELECTOR_WIDTH)
        self.selectors.add(sel.id)
        return sel

    def _aux(self, width: int):
        self.n_aux += 1
        leaf = self.lw.leaf("aux#%d" % self.n_aux, width, "aux", "")
        self.aux_seq[leaf.id] = len(self.aux_seq)
        return leaf

    def _key(self, leaf_id: int):
        """A leaf's identity across repeated constructions (run): its id, or
        a generated leaf's ordinal."""
        k = self.aux_seq.get(leaf_id)
        return leaf_id if k is None else -1 - k

    def _define(self, atoms) -> int:
        n = 0
        for x in atoms:
            if x.op == I.EQ:
                p, q = x.args
                done = False
                for leaf, e in ((p, q), (q, p)):
                    if leaf.op == I.LEAF and self._try_define(leaf, e):
                        done = True
                        break
                if not done:
                    # ite(c, leaf, y) = e (also nested: a first-match table
                    # read ite(k = k0, v0, ite(k = k1, v1, leaf))): the leaf's
                    # value e suffices on the path that reaches it
                    for side, e in ((p, q), (q, p)):
                        for arm in self._ite_leaves(side):
                            if self._try_define(arm, e):
                                done = True
                                break
                        if done:
                            break
                n += done
            elif x.op == I.OR and x.width == 1 and x.id not in self.or_seen:
                self.or_seen.add(x.id)           # the same or splits the same way again
                n += self._domain(x) or self._branches(x)
        return n

    def _ranges(self, atoms) -> int:
        """A leaf confined to a narrow interval (and / or fixed low bits):
        ``leaf = base + (aux << j)`` with a fresh ``aux`` sized to the
        interval (``keccak_function_manager``'s hash intervals:
        ``lower <= f(x) < upper, f(x) % 64 = 0``)."""
        info: Dict[int, list] = {}
        for x in atoms:
            b = self._bound(x)
            if b is not None and b[0].op == I.LEAF:
                e, lo, hi, _ = b
                r = info.setdefault(e.id, [e, 0, _mask(e.width), 0, 0])
                r[1], r[2] = max(r[1], lo), min(r[2], hi)
            elif x.op == I.EQ:
                a, k = x.args
                if a.op == I.CONST:
                    a, k = k, a
                if a.op == I.EXTRACT and a.imm == 0 and a.args[0].op == I.LEAF and \
                        k.op == I.CONST:
                    leaf = a.args[0]
                    r = info.setdefault(leaf.id, [leaf, 0, _mask(leaf.width), 0, 0])
                    if a.width > r[3]:
                        r[3], r[4] = a.width, k.imm
        n = 0
        for leaf, lo, hi, j, res in info.values():
            if leaf.id in self.repl or lo > hi or (not j and lo == 0 and hi == _mask(leaf.width)):
                continue
            base = ((lo >> j) << j) | res
            if base < lo:
                base += 1 << j
            if base > hi:
                continue
            room = ((hi - base) >> j) + 1       # values base + t * 2^j, t < room
            # a selector a conjunct confines commits to that branch
            a = 0 if leaf.id in self.selectors else room.bit_length() - 1
            lw = self.lw
            e = lw.const(base, leaf.width)
            if a > 0:
                aux = self._aux(a)
                step = aux if not j else lw.mk(I.CONCAT, a + j, (aux, lw.const(0, j)), j)
                e = lw.mk(I.ADD, leaf.width, (e, step)) if base else step
            n += self._try_define(leaf, e)
        return n

    def _branches(self, x) -> int:
        """An ``or`` of a few disjuncts: each disjunct's definitions, merged
        per leaf by a fresh selector (each candidate commits to one
        disjunct; a leaf a disjunct leaves free keeps a generated value)."""
        disj, stack = [], [x]
        while stack:
            y = stack.pop()
            if y.op == I.OR and y.width == 1:
                stack.extend(reversed(y.args))
            else:
                disj.append(y)
        if len(disj) > MAX_BRANCHES or self.n_branch >= MAX_OR:
            return 0
        saved, unsat = dict(self.repl), self.unsat
        per: List[Dict[int, object]] = []
        for d in disj:
            self.unsat = False
            atoms = self._atoms(d, _Overlay(self._memo))
            if self.unsat:
                per.append({})
                continue
            self._define(atoms)
            self._ranges(atoms)
            per.append({k: v for k, v in self.repl.items() if k not in saved})
            self.repl = dict(saved)
            self._dm = None
        self.unsat = unsat
        leaves = {}
        for defs in per:
            for k in defs:
                leaves.setdefault(k, None)
        if not leaves:
            return 0
        self.n_branch += 1
        lw = self.lw
        by_id = self.leaf_node
        sel = self._selector()
        span = 1 << SELECTOR_WIDTH
        n = 0
        for k in leaves:
            leaf = by_id[k]
            d = self.depth.get(k, 0)
            if d >= BRANCH_DEPTH:
                continue                         # (else every pass splits the same or)
            free = None
            arms = []
            for defs in per:
                e = defs.get(k)
                if e is None:
                    if free is None:
                        free = self._aux(leaf.width)
                        self.depth[free.id] = d + 1
                    e = free
                arms.append(e)
            e = arms[-1]
            for i in reversed(range(len(arms) - 1)):
                t = lw.const(span * (i + 1) // len(arms), SELECTOR_WIDTH)
                e = lw.mk(I.ITE, leaf.width, (lw.mk(I.ULT, SELECTOR_WIDTH, (sel, t)), arms[i], e))
            n += self._try_define(leaf, e)
        return n

    def _abi_offsets(self) -> list:
        """Symbolic table keys ``y + c`` whose base ``y`` is not constant
        (calldata read at an ABI offset that is itself a calldata word:
        ``calldata.py:219-232`` under a dynamic parameter) get ``y``
        pinned the way the ABI lays out dynamic data: right after the
        table's constant-key reads, 32-aligned, in order of first use —
        ``y = K`` atoms for the definition passes."""
        out = []
        for name, ents in self.lw.arg_entries.items():
            ck = self.lw.table_ckeys.get(name)
            if not ck or len(ents[0][0]) != 1:
                continue
            spans: Dict[int, list] = {}
            memo: Dict[int, object] = {}
            for key, _ in ents:
                k = self.rewrite(key[0], memo)
                y, c = (k.args[0], k.args[1].imm) if k.op == I.ADD and \
                    k.args[1].op == I.CONST else (k, 0)
                if y.op == I.CONST or c >> 32 or not self._reads_own(y, name):
                    continue
                r = spans.setdefault(y.id, [y, c, c])
                r[1], r[2] = min(r[1], c), max(r[2], c)
            nxt = max(ck) + 1
            for y, lo, hi in spans.values():
                base = -(-(nxt - lo) // 32) * 32           # first read lands past nxt
                out.append(self.lw.mk(I.EQ, y.width, (y, self.lw.const(base, y.width))))
                nxt = base + hi + 1
        return out

    def _joint_bounds(self, atoms):
        """The intersected bounds of every non-leaf expression bounded by
        two or more atoms, split (atoms to process one by one)."""
        groups: Dict[int, list] = {}
        for a in atoms:
            b = self._bound(a)
            if b is None or b[0].op in (I.LEAF, I.CONST):
                continue
            e, lo, hi, w = b
            g = groups.setdefault(e.id, [e, 0, _mask(w), w, 0])
            g[1], g[2], g[4] = max(g[1], lo), min(g[2], hi), g[4] + 1
        parts = []
        for e, lo, hi, w, k in groups.values():
            if k >= 2 and lo <= hi and (e.id, lo, hi) not in self.joint_done:
                self.joint_done.add((e.id, lo, hi))
                # split with both limits at once (separate atoms would be
                # split apart again)
                sp = self._split_bound(e, lo, hi, w) if e.op in (I.CONCAT, I.ITE, I.MUL) \
                    else None
                parts += sp if sp is not None else self._mk_bound(e, lo, hi, w)
        return parts

    @staticmethod
    def _is_wrap_test(r) -> bool:
        """``not bvumul_noovfl(a, b)`` or the carry test ``a + b < a``."""
        x = r
        while x.op == I.AND and x.width == 1 and len(x.args) == 2 and x.args[0].op == I.CONST:
            x = x.args[1]
        if x.op == I.NOT and x.width == 1 and x.args[0].op == I.UMULNO:
            return True
        return x.op == I.ULT and x.args[0].op == I.ADD and x.args[1] in x.args[0].args

    def _reads_own(self, y, name: str) -> bool:
        """``y`` is built from the table's own cells (and its size): an
        offset word read from the calldata it indexes."""
        own = False
        for li in _bit_indices(self._dep(y)):
            leaf = self.lw.leaves[li]
            if leaf.source == name:
                own = True
            elif not leaf.name.endswith("calldatasize"):
                return False
        return own

    def _culprit(self, r) -> Optional[int]:
        """The definition (index into the insertion-ordered definitions) that
        completes root ``r``'s folding to false: the shortest prefix under
        which it folds to false ends with it.  None when ``r`` is false with
        no definitions at all."""
        items = list(self.repl.items())
        saved = self.repl

        def false_under(m: int) -> bool:
            self.repl = dict(items[:m])
            self._dm = None
            return _is_false(self.rewrite(r, {}))
        lo, hi = 0, len(items)                   # false_under(hi) holds
        if false_under(0):
            lo = None
        else:
            while hi - lo > 1:                   # false_under(lo) is False
                mid = (lo + hi) // 2
                if false_under(mid):
                    hi = mid
                else:
                    lo = mid
        self.repl = saved
        self._dm = None
        return None if lo is None else hi - 1

    def run(self, roots):
        # new nodes are born with their latest operand (ir._schedule places
        # them there), not after the whole query
        saved_birth, self.lw.birth = self.lw.birth, 0
        pins = self._abi_offsets()
        if pins:
            self._define(self._atoms(self.lw.mk(I.AND, 1, tuple(pins)) if len(pins) > 1
                                     else pins[0], {}))
        # the overflow tests first (the integer module's check is the
        # query's last constraint; its wrap-around choice must win over the
        # bounds the path constraints put on the same operands)
        order = sorted(roots, key=lambda r: not self._is_wrap_test(r))
        base = list(self.repl.items())
        for attempt in range(MAX_REFUSALS + 1):
            dead, at_pass = self._passes(order)
            if dead is None:
                break
            # a root folded to false under the construction.  When the
            # definition that completed it came from the overflow test (the
            # module's check: a SafeMath check whose require is on the path)
            # or the first pass, that is the query's own conditions meeting:
            # the group needs no program beyond that root
            # (model._ground_value).  Otherwise it is heuristic commits
            # conflicting (the C3 overflow checks after an approve: a
            # table-arm commit and a branch split): refuse the definition
            # that completed the false root and construct again, up to
            # MAX_REFUSALS times
            k = self._culprit(dead) if at_pass and attempt < MAX_REFUSALS else None
            if k is not None and list(self.repl)[k] in self.wrap_defs:
                k = None                         # the check's own choice: not refused
            if k is None:
                self.dead = True
                self.lw.birth = saved_birth
                return [self.rewrite(dead, self._memo)], {}
            self.refused.add(self._key(list(self.repl)[k]))
            self.repl = dict(base)
            self._dm = None
            self.or_seen = set()
            self.joint_done = set()
            self.n_branch = 0
            self.aux_seq = {}
            self.wrap_defs = set()
            self.depth = {}
        memo = self._memo
        new_roots = [self.rewrite(r, memo) for r in roots]
        by_id = self.leaf_node
        defs = {by_id[k].imm: self.rewrite(e, memo) for k, e in self.repl.items()}
        self.lw.birth = saved_birth
        return new_roots, defs

    def _passes(self, order):
        """The definition passes: (the first root that folds to false, the
        pass it folded in), or (None, None)."""
        # one memo for the whole run: rewrite drops the entries a new
        # definition reaches (later roots see the new definitions folded)
        memo: Dict[int, object] = {}
        self._memo = memo
        for at_pass in range(PASSES):
            found = 0
            every = []
            for r in order:
                self._wrap_ctx = self._is_wrap_test(r)
                atoms = self._atoms(r, memo)
                rr = self.rewrite(r, memo)
                if rr.op == I.CONST and not rr.imm & 1:
                    self._wrap_ctx = False
                    return r, at_pass
                every += atoms
                found += self._define(atoms)
            self._wrap_ctx = False
            # intervals from the bounds of all conjuncts together: per
            # expression (x >= 2 from one constraint, x <= 2 from another make
            # x = 2 — through a concat, its low byte), then per leaf
            if found:
                every = [self.rewrite(a, memo) for a in every]
            extra = []
            for part in self._joint_bounds(every):     # one by one: a violated
                extra += self._atoms(part, memo)      # part must not hide the rest
            if extra:
                found += self._define(extra)
                every += extra
            found += self._ranges(every)
            if not found:
                break
        return None, None
