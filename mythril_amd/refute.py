"""Host-side refutation of a query group before any compile or launch.

A cold ``get_model`` miss on an unsatisfiable query pays the search compile
and a launch before z3 is asked (C3, 62 of 64 queries UNSAT by
construction).  Most of those contradictions are local: SafeMath's
``require`` on two terms and the detection module's check on the SAME two
terms (``integer.py:274-280`` poses ``ULT(a, b)`` for a subtraction that the
contract guarded with ``require(b <= a)``; an addition guarded with
``require(a + b >= a)`` is checked with z3's carry shape ``a + b <u a``).
Hash-consing makes "the same term" node identity, so the contradiction is
visible in the group's atoms without lowering anything.

The rule is exact order reasoning per term pair: for terms x, y the unsigned
(and, separately, the signed) relation is one of LT / EQ / GT; every atom over
(x, y) — ``bvult``/``bvule``/``bvugt``/``bvuge``, their signed forms, ``=``,
``distinct``, ``not`` of any, ``or`` of atoms over the same pair (LASER's
``UGE = Or(UGT, ==)``, ``bitvec_helper.py``), LASER's JUMPI / ISZERO shape
``If(c, 1, 0) == 0`` (``instructions.py``) — restricts the set of relations
the pair can be in; conjuncts intersect.  An empty set is a contradiction.
A term equal to a numeral is also evaluated against the other numerals it is
compared with.  Every step is an equivalence or an over-approximation of the
satisfying set, so a refuted group is unsatisfiable; anything the rule does
not understand constrains nothing.

Refutation only moves time: the query still goes to z3, which alone
concludes UNSAT (``mythril/support/model.py:44-49``; ``model.gpu_search``).
"""

from typing import Dict, List, Optional, Sequence, Tuple

from .smt import node as N

LT, EQ, GT = 1, 2, 4
ALL = LT | EQ | GT
_REL = {"bvult": ("u", LT), "bvule": ("u", LT | EQ), "bvugt": ("u", GT), "bvuge": ("u", GT | EQ),
        "bvslt": ("s", LT), "bvsle": ("s", LT | EQ), "bvsgt": ("s", GT), "bvsge": ("s", GT | EQ)}
# atoms examined per group before the rule gives up (bounds its latency)
MAX_ATOMS = 4096


def _mirror(m: int) -> int:
    """The relation of (y, x) given that of (x, y)."""
    return ((m & LT) << 2) | (m & EQ) | ((m & GT) >> 2)


# An atom: (domain, x, y, mask) with x.id <= y.id; domain "u" (unsigned
# order), "s" (signed order) or "e" (equality: the same relation in both)
Atom = Tuple[str, N.Node, N.Node, int]


def _pair(dom: str, x: N.Node, y: N.Node, m: int) -> Atom:
    return (dom, x, y, m) if x.id <= y.id else (dom, y, x, _mirror(m))


def _bit(n: N.Node) -> Optional[bool]:
    """ite(c, 1, 0): True; ite(c, 0, 1): False (the constant arms LASER's
    Bool-to-BitVec conversion uses); else None."""
    if n.op != "ite" or len(n.args) != 3:
        return None
    t, e = n.args[1], n.args[2]
    if t.op == "bvnum" and e.op == "bvnum":
        if t.params[0] == 1 and e.params[0] == 0:
            return True
        if t.params[0] == 0 and e.params[0] == 1:
            return False
    return None


def _atom(c: N.Node, neg: bool) -> Optional[Atom]:
    """One relation atom equivalent to c (negated when neg), or None."""
    while c.op == "not":
        c, neg = c.args[0], not neg
    op = c.op
    if op in _REL and len(c.args) == 2:
        dom, m = _REL[op]
        return _pair(dom, c.args[0], c.args[1], (ALL & ~m) if neg else m)
    if op in ("=", "distinct") and len(c.args) == 2 and c.args[0].is_bv():
        x, y = c.args
        eq = (op == "=") != neg
        # If(c, 1, 0) == k: the condition itself (LASER's JUMPI / ISZERO)
        for u, k in ((x, y), (y, x)):
            b = _bit(u)
            if b is not None and k.op == "bvnum" and k.params[0] in (0, 1):
                inner = b == bool(k.params[0])
                return _atom(u.args[0], not (inner == eq))
        return _pair("e", x, y, EQ if eq else LT | GT)
    if (op == "or" and not neg) or (op == "and" and neg):
        # a disjunction of atoms over one pair in one order domain
        acc = None
        for a in c.args:
            t = _atom(a, neg)
            if t is None:
                return None
            if acc is None:
                acc = t
                continue
            if t[1] is not acc[1] or t[2] is not acc[2]:
                return None
            dom = acc[0] if t[0] == "e" else t[0] if acc[0] == "e" else acc[0]
            if acc[0] != "e" and t[0] != "e" and acc[0] != t[0]:
                return None
            acc = (dom, acc[1], acc[2], acc[3] | t[3])
        return acc
    return None


def _conjuncts(roots: Sequence[N.Node]) -> List[Tuple[N.Node, bool]]:
    """The (node, negated) conjuncts of the roots: ``and`` and ``not or``
    flattened, double negations dropped."""
    out, stack = [], [(r, False) for r in reversed(list(roots))]
    while stack and len(out) < MAX_ATOMS:
        c, neg = stack.pop()
        while c.op == "not":
            c, neg = c.args[0], not neg
        if (c.op == "and" and not neg) or (c.op == "or" and neg):
            stack.extend((a, neg) for a in reversed(c.args))
            continue
        b = None
        if c.op == "=" and len(c.args) == 2:
            for u, k in ((c.args[0], c.args[1]), (c.args[1], c.args[0])):
                bb = _bit(u)
                if bb is not None and k.op == "bvnum" and k.params[0] in (0, 1):
                    b = (u.args[0], neg != (bb != bool(k.params[0])))
        if b is not None:                 # If(c, 1, 0) == k: descend into c
            stack.append(b)
            continue
        out.append((c, neg))
    return out


def _signed(v: int, w: int) -> int:
    return v - (1 << w) if v >> (w - 1) else v


def _holds(dom: str, a: int, b: int, w: int, m: int) -> bool:
    if dom == "s":
        a, b = _signed(a, w), _signed(b, w)
    rel = LT if a < b else GT if a > b else EQ
    return bool(rel & m)


def _carry(c: N.Node) -> Optional[Tuple[N.Node, N.Node, int]]:
    """z3's BVAddNoOverflow carry shape ``extract(w, w, zext1(a) + zext1(b))``
    (the unsigned carry out of a + b): (a, b, carry value compared with)."""
    if c.op != "=" or len(c.args) != 2:
        return None
    for e, k in ((c.args[0], c.args[1]), (c.args[1], c.args[0])):
        if e.op == "extract" and k.op == "bvnum" and e.width == 1 and e.args[0].op == "bvadd":
            s = e.args[0]
            w = s.width - 1
            if e.params == (w, w) and len(s.args) == 2 and all(
                    z.op == "zero_extend" and z.params == (1,) for z in s.args):
                return s.args[0].args[0], s.args[1].args[0], k.params[0]
    return None


def _overflow_atoms(a: N.Node, b: N.Node, carry: bool) -> List[Atom]:
    """Atoms equivalent to "a + b carries" (or not): with s = a + b mod 2^w,
    the carry is s <u a, equally s <u b, for either operand order of the
    sum (only sums that exist: a new node could not occur in another atom)."""
    out = []
    for x, y in ((a, b), (b, a)):
        s = N.find("bvadd", N.BV, a.width, (x, y))
        if s is None:
            continue
        for t in (a, b):
            out.append(_pair("u", s, t, LT if carry else GT | EQ))
    return out


def refuted(roots: Sequence[N.Node]) -> bool:
    """True when the conjunction of ``roots`` is unsatisfiable by the pair
    and interval rules (never for a satisfiable one)."""
    sets: Dict[Tuple[int, int], List] = {}          # (x.id, y.id) -> [x, y, u, s]
    overflow: List[Tuple[str, N.Node, N.Node]] = []  # ("add" | "mul", a, b): must overflow
    no_overflow: List[Tuple[str, N.Node, N.Node]] = []

    def note(a: Atom) -> bool:
        dom, x, y, m = a
        if x is y:
            return not (m & EQ)            # x < x, x != x
        st = sets.setdefault((x.id, y.id), [x, y, ALL, ALL])
        if dom in ("u", "e"):
            st[2] &= m
        if dom in ("s", "e"):
            st[3] &= m
        return False

    for c, neg in _conjuncts(roots):
        if c.op == "false" and not neg or c.op == "true" and neg:
            return True
        cy = _carry(c)
        if cy is not None:
            a, b, k = cy
            carry = (k == 1) != neg
            (overflow if carry else no_overflow).append(("add", a, b))
            if any(note(t) for t in _overflow_atoms(a, b, carry)):
                return True
            continue
        if c.op == "bvumul_noovfl" and len(c.args) == 2:
            (overflow if neg else no_overflow).append(("mul", c.args[0], c.args[1]))
            continue
        t = _atom(c, neg)
        if t is not None and note(t):
            return True
    if set(overflow) & set(no_overflow):
        return True
    # per pair: the two orders agree on equality
    for st in sets.values():
        x, y, u, s = st
        if not (u & EQ) or not (s & EQ):             # x != y in one order: in both
            u, s = u & ~EQ, s & ~EQ
        st[2], st[3] = u, s
        if not u or not s:
            return True
        if x.op == "bvnum" and y.op == "bvnum":
            w = x.width
            if not (_holds("u", x.params[0], y.params[0], w, u) and
                    _holds("s", x.params[0], y.params[0], w, s)):
                return True
    # unsigned intervals of terms compared with numerals
    lo: Dict[int, int] = {}
    hi: Dict[int, int] = {}
    for x, y, u, s in sets.values():
        for t, k, m in ((x, y, u), (y, x, _mirror(u))):
            if k.op != "bvnum" or t.op == "bvnum":
                continue
            v, top = k.params[0], (1 << t.width) - 1
            l, h = lo.get(t.id, 0), hi.get(t.id, top)
            if not (m & (LT | EQ)):
                l = max(l, v + 1)
            elif not (m & LT):
                l = max(l, v)
            if not (m & (GT | EQ)):
                h = min(h, v - 1)
            elif not (m & GT):
                h = min(h, v)
            if m == LT | GT and l == h == v:
                return True
            if l > h:
                return True
            lo[t.id], hi[t.id] = l, h
    for kind, a, b in overflow + no_overflow:
        w = a.width
        la, ha = lo.get(a.id, 0), hi.get(a.id, (1 << w) - 1)
        lb, hb = lo.get(b.id, 0), hi.get(b.id, (1 << w) - 1)
        if kind == "add":
            most, least = ha + hb, la + lb
        else:
            most, least = ha * hb, la * lb
        must = (kind, a, b) in overflow
        if must and most < (1 << w):
            return True                       # cannot overflow
        if not must and least >= (1 << w):
            return True                       # always overflows
    return False
