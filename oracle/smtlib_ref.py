"""ORACLE — test infrastructure only (never imported by the product path).

CPU restatement of what the reference's hot path computes when it asks z3 to
evaluate a ``get_model`` constraint DAG under a candidate assignment
(``z3.Model.eval`` / ``substitute``+``simplify``, reached from
``mythril/support/model.py:15-49`` through
``mythril/laser/smt/solver/solver.py:47-64`` and ``laser/smt/model.py:44-59``).

The arithmetic itself lives in the third-party dependency **z3-solver**
(``requirements.txt:30``/``setup.py:30``: ``z3-solver>=4.8.5.0``, unpinned, not
vendored under /root/reference and not installed in this image).  What z3
implements here is the SMT-LIB 2.6 ``FixedSizeBitVectors`` theory with
``rewriter.hi_div0=true`` (its default), i.e.:

* ``bvudiv a 0 = 2^w-1``, ``bvurem a 0 = a``; ``bvsdiv``/``bvsrem``/``bvsmod``
  are defined from ``bvudiv``/``bvurem`` on magnitudes exactly as the SMT-LIB
  standard writes them (so ``bvsdiv a 0 = a<0 ? 1 : -1``, ``bvsrem a 0 = a``,
  ``bvsmod a 0 = a``, ``bvsdiv(-2^(w-1), -1) = -2^(w-1)``);
* shifts by ``>= w`` give 0 (``bvashr``: all sign bits);
* ``concat a b`` puts ``a`` in the high bits; ``extract`` bounds are inclusive;
* ``bvumul_noovfl a b <=> a*b < 2^w``;
* arrays/UFs are interpreted as z3 models print them: a finite list of
  ``(key -> value)`` entries tried in order, then an ``else`` value;
  ``select (store A i v) j = (i == j ? v : select A j)``; ``K`` is constant.

Python integers make every definition a one-liner, so this module is the
arbiter used to pin the C oracle (``oracle/evalref.c``) and the HIP engine.
Parity pinning: see ``tests/test_oracle_golden.py`` (EIP-145 shift vectors from
``tests/instructions/{shl,shr,sar}_test.py``, VMTest arithmetic/bitwise
post-states from ``tests/laser/evm_testsuite/VMTests``, Keccak-256 KATs from
``vmSha3Test``).
"""

from __future__ import annotations

from typing import Dict, List, Tuple

Table = Tuple[List[Tuple[int, int]], int]


class Assignment:
    """A candidate model: BV/Bool variables, free-array and UF tables."""

    def __init__(self, vars: Dict[str, int] = None, arrays: Dict[str, Table] = None,
                 funcs: Dict[str, Table] = None):
        self.vars = dict(vars or {})
        self.arrays = dict(arrays or {})
        self.funcs = dict(funcs or {})


def _mask(w: int) -> int:
    return (1 << w) - 1


def _signed(x: int, w: int) -> int:
    return x - (1 << w) if x >> (w - 1) else x


def bvudiv(a: int, b: int, w: int) -> int:
    return _mask(w) if b == 0 else a // b


def bvurem(a: int, b: int, w: int) -> int:
    return a if b == 0 else a % b


def bvneg(a: int, w: int) -> int:
    return (-a) & _mask(w)


def bvsdiv(s: int, t: int, w: int) -> int:
    ms, mt = s >> (w - 1), t >> (w - 1)
    if not ms and not mt:
        return bvudiv(s, t, w)
    if ms and not mt:
        return bvneg(bvudiv(bvneg(s, w), t, w), w)
    if not ms and mt:
        return bvneg(bvudiv(s, bvneg(t, w), w), w)
    return bvudiv(bvneg(s, w), bvneg(t, w), w)


def bvsrem(s: int, t: int, w: int) -> int:
    ms, mt = s >> (w - 1), t >> (w - 1)
    if not ms and not mt:
        return bvurem(s, t, w)
    if ms and not mt:
        return bvneg(bvurem(bvneg(s, w), t, w), w)
    if not ms and mt:
        return bvurem(s, bvneg(t, w), w)
    return bvneg(bvurem(bvneg(s, w), bvneg(t, w), w), w)


def bvsmod(s: int, t: int, w: int) -> int:
    ms, mt = s >> (w - 1), t >> (w - 1)
    abs_s = bvneg(s, w) if ms else s
    abs_t = bvneg(t, w) if mt else t
    u = bvurem(abs_s, abs_t, w)
    if u == 0:
        return u
    if not ms and not mt:
        return u
    if ms and not mt:
        return (bvneg(u, w) + t) & _mask(w)
    if not ms and mt:
        return (u + t) & _mask(w)
    return bvneg(u, w)


def bvshl(a: int, b: int, w: int) -> int:
    return 0 if b >= w else (a << b) & _mask(w)


def bvlshr(a: int, b: int, w: int) -> int:
    return 0 if b >= w else a >> b


def bvashr(a: int, b: int, w: int) -> int:
    sa = _signed(a, w)
    if b >= w:
        return _mask(w) if sa < 0 else 0
    return (sa >> b) & _mask(w)


def _lookup(table: Table, key: int) -> int:
    entries, default = table
    for k, v in entries:
        if k == key:
            return v
    return default


class _ArrayVal:
    """Functional array value: base table/constant plus a store overlay."""

    __slots__ = ("base_table", "const", "stores")

    def __init__(self, base_table=None, const=None, stores=()):
        self.base_table = base_table
        self.const = const
        self.stores = stores      # tuple of (idx, val), newest last

    def get(self, idx: int) -> int:
        for k, v in reversed(self.stores):
            if k == idx:
                return v
        if self.const is not None:
            return self.const
        return _lookup(self.base_table, idx)


def evaluate(roots, asg: Assignment, cache: dict = None) -> list:
    """Evaluate each root node under ``asg``; Bool → 0/1, BV → int,
    Array → ``_ArrayVal``.  Iterative over the DAG (shared sub-terms once)."""
    from mythril_amd.smt.node import topo_order  # node structure only

    val = {} if cache is None else cache
    for n in topo_order(roots):
        if n.id in val:
            continue
        op, w = n.op, n.width
        a = [val[x.id] for x in n.args]
        if op == "bvnum":
            r = n.params[0]
        elif op == "true":
            r = 1
        elif op == "false":
            r = 0
        elif op == "var":
            if n.params[0] not in asg.vars:
                raise KeyError("assignment lacks variable %r" % n.params[0])
            r = asg.vars[n.params[0]] & _mask(w)
        elif op == "array":
            r = _ArrayVal(base_table=asg.arrays[n.params[0]])
        elif op == "K":
            r = _ArrayVal(const=a[0])
        elif op == "store":
            r = _ArrayVal(a[0].base_table, a[0].const, a[0].stores + ((a[1], a[2]),))
        elif op == "select":
            r = a[0].get(a[1])
        elif op == "apply":
            r = _lookup(asg.funcs[n.params[0]], a[0])
        elif op == "bvadd":
            r = sum(a) & _mask(w)
        elif op == "bvmul":
            r = 1
            for x in a:
                r = (r * x) & _mask(w)
        elif op == "bvsub":
            r = (a[0] - a[1]) & _mask(w)
        elif op == "bvneg":
            r = bvneg(a[0], w)
        elif op == "bvand":
            r = _mask(w)
            for x in a:
                r &= x
        elif op == "bvor":
            r = 0
            for x in a:
                r |= x
        elif op == "bvxor":
            r = 0
            for x in a:
                r ^= x
        elif op == "bvnot":
            r = a[0] ^ _mask(w)
        elif op == "bvudiv":
            r = bvudiv(a[0], a[1], w)
        elif op == "bvurem":
            r = bvurem(a[0], a[1], w)
        elif op == "bvsdiv":
            r = bvsdiv(a[0], a[1], w)
        elif op == "bvsrem":
            r = bvsrem(a[0], a[1], w)
        elif op == "bvsmod":
            r = bvsmod(a[0], a[1], w)
        elif op == "bvshl":
            r = bvshl(a[0], a[1], w)
        elif op == "bvlshr":
            r = bvlshr(a[0], a[1], w)
        elif op == "bvashr":
            r = bvashr(a[0], a[1], w)
        elif op == "concat":
            r = 0
            for x, arg in zip(a, n.args):
                r = (r << arg.width) | x
        elif op == "extract":
            hi, lo = n.params
            r = (a[0] >> lo) & _mask(hi - lo + 1)
        elif op == "zero_extend":
            r = a[0]
        elif op == "sign_extend":
            r = _signed(a[0], n.args[0].width) & _mask(w)
        elif op == "=":
            r = int(_eqv(a[0], a[1], n.args[0]))
        elif op == "distinct":
            r = int(len(set(a)) == len(a)) if not n.args[0].is_array() else \
                int(not _eqv(a[0], a[1], n.args[0]))
        elif op == "ite":
            r = a[1] if a[0] else a[2]
        elif op == "and":
            r = int(all(a))
        elif op == "or":
            r = int(any(a))
        elif op == "xor":
            r = a[0] ^ a[1]
        elif op == "not":
            r = 1 - a[0]
        elif op == "=>":
            r = int((not a[0]) or a[1])
        elif op in ("bvult", "bvule", "bvugt", "bvuge"):
            x, y = a
            r = int({"bvult": x < y, "bvule": x <= y, "bvugt": x > y, "bvuge": x >= y}[op])
        elif op in ("bvslt", "bvsle", "bvsgt", "bvsge"):
            ww = n.args[0].width
            x, y = _signed(a[0], ww), _signed(a[1], ww)
            r = int({"bvslt": x < y, "bvsle": x <= y, "bvsgt": x > y, "bvsge": x >= y}[op])
        elif op == "bvumul_noovfl":
            r = int(a[0] * a[1] < (1 << n.args[0].width))
        else:
            raise NotImplementedError("oracle: op %s" % op)
        val[n.id] = r
    return [val[r.id] for r in roots]


def _eqv(x, y, n) -> bool:
    if n.is_array():
        raise NotImplementedError("array extensionality is outside the hot-path vocabulary")
    return x == y


def eval_constraints(constraints, asg: Assignment) -> int:
    """Conjunction of Bool constraint nodes → 0/1 (the ``get_model`` root)."""
    vals = evaluate(list(constraints), asg)
    return int(all(vals))
