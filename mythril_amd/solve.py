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
(``laser/ethereum/function_managers/keccak_function_manager.py``'s
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


_PREDICATES = (I.EQ, I.ULT, I.ULE, I.SLT, I.SLE, I.UMULNO)


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
        self.clean: set = set()                  # ids of rewrite results
        self.leaf_imm: Dict[int, int] = {}       # defined LEAF id -> leaf index
        self._dm = None                          # bit set of the defined leaves
        # LEAF id -> generation of a branch's stand-in for an undefined value
        # (a stand-in may be split again by a later ``or``, to BRANCH_DEPTH)
        self.depth: Dict[int, int] = {}
        self.unsat = False

    # -- rewriting -------------------------------------------------------------
    def _fold(self, x, args):
        lw, op = self.lw, x.op
        if op == I.EQ:
            a, b = args
            if a is b:
                return self.one
            if a.op == I.CONST and b.op == I.CONST:
                return self.one if a.imm == b.imm else self.zero
        elif op in (I.ULT, I.ULE) and all(a.op == I.CONST for a in args):
            a, b = args[0].imm, args[1].imm
            return self.one if (a < b if op == I.ULT else a <= b) else self.zero
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
        its own result — the walk does not enter it."""
        dm = self._defmask()
        clean, dep = self.clean, self._dep
        stack = [(n, False)]
        while stack:
            x, done = stack.pop()
            if x.id in memo:
                continue
            if x.op == I.LEAF:
                e = self.repl.get(x.id)
                if e is None:
                    memo[x.id] = x
                elif e.id in memo:
                    memo[x.id] = memo[e.id]
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
                stack.extend((a, False) for a in x.args if a.id not in memo)
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
                return [c, self._eq(p, k)] if q.imm != k else [self._eq(p, k)]
            if p.op == I.CONST:
                return [self._not(c), self._eq(q, k)] if p.imm != k else [self._eq(q, k)]
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
            if y.op == I.ITE and (y.args[1].op == I.CONST or y.args[2].op == I.CONST):
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
                out.append(x)
                if y.op == I.UMULNO and y.args[1].op != I.CONST:
                    # a * b >= 2^w (BVMulNoOverflow negated): b = 2^w - 1
                    # suffices for every a > 1
                    b_ = y.args[1]
                    stack.append(self.rewrite(self._eq(b_, _mask(b_.width)), memo))
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
            if b is not None and b[0].op == I.ITE:
                parts = self._split_bound(*b)
                if parts is not None:
                    stack.extend(self.rewrite(p, memo) for p in parts)
                    continue
            out.append(x)
        return out

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

    def _split_bound(self, e, lo, hi, w) -> Optional[list]:
        """``lo <= ite(c, k, y) <= hi``: ``y`` in range suffices when ``k`` is
        (else ``not c`` is needed too)."""
        c, p, q = e.args
        if p.op == I.CONST and q.op != I.CONST:
            inside = lo <= p.imm <= hi
            return self._mk_bound(q, lo, hi, w) + ([] if inside else [self._not(c)])
        if q.op == I.CONST and p.op != I.CONST:
            inside = lo <= q.imm <= hi
            return self._mk_bound(p, lo, hi, w) + ([] if inside else [c])
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
        if e.width > leaf.width and not (e.op == I.CONST and e.imm >> leaf.width == 0):
            return False
        if self._depends(e, leaf):
            return False
        self.repl[leaf.id] = e
        self.leaf_imm[leaf.id] = leaf.imm
        self._dm = None
        return True

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
        return self.lw.leaf("aux#%d" % self.n_aux, width, "aux", "")

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
                    # ite(c, leaf, y) = e: the leaf's value e suffices when c
                    for side, e in ((p, q), (q, p)):
                        if side.op == I.ITE:
                            for arm in side.args[1:]:
                                if arm.op == I.LEAF and self._try_define(arm, e):
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
            atoms = self._atoms(d, {})
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
        by_id = {n.id: n for n in lw.table.values() if n.op == I.LEAF}
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

    def run(self, roots):
        # new nodes are born with their latest operand (ir._schedule places
        # them there), not after the whole query
        saved_birth, self.lw.birth = self.lw.birth, 0
        for _ in range(PASSES):
            memo: Dict[int, object] = {}
            found = 0
            every = []
            for r in roots:
                atoms = self._atoms(r, memo)
                every += atoms
                k = self._define(atoms)
                if k:                   # later roots see the new definitions folded
                    memo = {}
                found += k
            # intervals from the bounds of all conjuncts together
            if found:
                memo = {}
                every = [self.rewrite(a, memo) for a in every]
            found += self._ranges(every)
            if not found:
                break
        memo = {}
        new_roots = [self.rewrite(r, memo) for r in roots]
        by_id = {n.id: n for n in self.lw.table.values() if n.op == I.LEAF}
        defs = {by_id[k].imm: self.rewrite(e, memo) for k, e in self.repl.items()}
        self.lw.birth = saved_birth
        return new_roots, defs
