"""Test infrastructure: a minimal stand-in for the z3 Python API surface that
mythril_amd/z3bridge.py uses (z3 is not installed here).  Expressions are
hash-consed applications with ``get_id``/``children``/``decl``/``params``/
``sort`` like z3's ``ExprRef``; declaration names and kinds follow z3's
(``bvadd``, ``if``, ``bvudiv_i``, ``extract`` with params, uninterpreted
constants and functions with ``Z3_OP_UNINTERPRETED``).  ``simplify`` of a
ground term evaluates it with the oracle (oracle/smtlib_ref.py) through the
bridge's own ``to_node``; ``Solver`` decides a query whose symbols are all
pinned by equalities.  Counters record how often ``children`` is called, so
tests can show the bridge's walks are linear in the DAG."""

from __future__ import annotations

from typing import Dict, List, Tuple

Z3_OP_UNINTERPRETED = 2051
Z3_OP_INTERPRETED = 1


class _Result:
    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return self.name


sat, unsat, unknown = _Result("sat"), _Result("unsat"), _Result("unknown")
CALLS = {"children": 0}


class Sort:
    def __init__(self, kind: str, size: int = 0, dom=None, rng=None):
        self.kind, self._size, self._dom, self._rng = kind, size, dom, rng

    def size(self):
        return self._size

    def domain(self):
        return self._dom

    def range(self):
        return self._rng

    def key(self):
        return (self.kind, self._size, self._dom.key() if self._dom else None,
                self._rng.key() if self._rng else None)


def BitVecSort(w):
    return Sort("bv", w)


BOOL = Sort("bool")


class FuncDecl:
    def __init__(self, name, kind, rng, params=(), dom=()):
        self._name, self._kind, self._rng, self._params, self._dom = name, kind, rng, tuple(params), dom

    def name(self):
        return self._name

    def kind(self):
        return self._kind

    def params(self):
        return list(self._params)

    def range(self):
        return self._rng

    def domain(self, i):
        return self._dom[i]

    def __call__(self, *args):
        return _mk(self, list(args), self._rng)


_TABLE: Dict[tuple, "Expr"] = {}


class Expr:
    def __init__(self, decl, args, sort, value=None, eid=0):
        self._decl, self._args, self._sort, self._value, self._id = decl, args, sort, value, eid

    # -- z3 ExprRef surface --------------------------------------------------
    def get_id(self):
        return self._id

    def children(self):
        CALLS["children"] += 1
        return list(self._args)

    def decl(self):
        return self._decl

    def params(self):
        return self._decl.params()

    def sort(self):
        return self._sort

    def size(self):
        return self._sort.size()

    def as_long(self):
        return self._value

    def __repr__(self):
        if self._value is not None:
            return "#%s" % self._value
        if not self._args:
            return self._decl.name()
        return "(%s %s)" % (self._decl.name(), " ".join(map(repr, self._args)))

    # -- operators (z3py BitVecRef semantics) ---------------------------------
    def _bin(self, name, other):
        return _op(name, self._sort, self, _lift(other, self))

    def __add__(self, o): return self._bin("bvadd", o)
    def __sub__(self, o): return self._bin("bvsub", o)
    def __mul__(self, o): return self._bin("bvmul", o)
    def __truediv__(self, o): return self._bin("bvsdiv", o)
    def __mod__(self, o): return self._bin("bvsmod", o)
    def __and__(self, o): return self._bin("bvand", o)
    def __or__(self, o): return self._bin("bvor", o)
    def __xor__(self, o): return self._bin("bvxor", o)
    def __lshift__(self, o): return self._bin("bvshl", o)
    def __rshift__(self, o): return self._bin("bvashr", o)
    def __invert__(self): return _op("bvnot", self._sort, self)
    def __neg__(self): return _op("bvneg", self._sort, self)
    def __lt__(self, o): return _op("bvslt", BOOL, self, _lift(o, self))
    def __le__(self, o): return _op("bvsle", BOOL, self, _lift(o, self))
    def __gt__(self, o): return _op("bvsgt", BOOL, self, _lift(o, self))
    def __ge__(self, o): return _op("bvsge", BOOL, self, _lift(o, self))

    def __eq__(self, o):  # noqa: D105 - z3 semantics: builds an equation
        return _op("=", BOOL, self, _lift(o, self))

    def __ne__(self, o):
        return _op("distinct", BOOL, self, _lift(o, self))

    __hash__ = object.__hash__


def _mk(decl, args, sort, value=None):
    key = (decl.name(), decl.kind(), tuple(decl.params()), tuple(a.get_id() for a in args),
           sort.key(), value)
    e = _TABLE.get(key)
    if e is None:
        e = Expr(decl, args, sort, value, len(_TABLE) + 1)
        _TABLE[key] = e
    return e


def _op(name, sort, *args, params=()):
    return _mk(FuncDecl(name, Z3_OP_INTERPRETED, sort, params), list(args), sort)


def _lift(o, like):
    return o if isinstance(o, Expr) else BitVecVal(o, like.size())


# -- constructors ---------------------------------------------------------------
def BitVecVal(v, w):
    w = w if isinstance(w, int) else w.size()
    return _mk(FuncDecl("bv", Z3_OP_INTERPRETED, BitVecSort(w)), [], BitVecSort(w), v % (1 << w))


def BoolVal(b):
    return _mk(FuncDecl("true" if b else "false", Z3_OP_INTERPRETED, BOOL), [], BOOL)


def BitVec(name, w):
    return _mk(FuncDecl(name, Z3_OP_UNINTERPRETED, BitVecSort(w)), [], BitVecSort(w))


def Bool(name):
    return _mk(FuncDecl(name, Z3_OP_UNINTERPRETED, BOOL), [], BOOL)


def Array(name, dom, rng):
    s = Sort("array", 0, dom, rng)
    return _mk(FuncDecl(name, Z3_OP_UNINTERPRETED, s), [], s)


def K(dom, v):
    s = Sort("array", 0, dom, v.sort())
    return _op("const", s, v)


def Store(a, i, v):
    return _op("store", a.sort(), a, i, v)


def Select(a, i):
    return _op("select", a.sort().range(), a, i)


def Function(name, dom, rng):
    return FuncDecl(name, Z3_OP_UNINTERPRETED, rng, dom=(dom,))


def UDiv(a, b): return _op("bvudiv", a.sort(), a, _lift(b, a))
def URem(a, b): return _op("bvurem", a.sort(), a, _lift(b, a))
def SRem(a, b): return _op("bvsrem", a.sort(), a, _lift(b, a))
def LShR(a, b): return _op("bvlshr", a.sort(), a, _lift(b, a))
def ULT(a, b): return _op("bvult", BOOL, a, _lift(b, a))
def ULE(a, b): return _op("bvule", BOOL, a, _lift(b, a))
def UGT(a, b): return _op("bvugt", BOOL, a, _lift(b, a))
def UGE(a, b): return _op("bvuge", BOOL, a, _lift(b, a))


def Concat(*a):
    return _op("concat", BitVecSort(sum(x.size() for x in a)), *a)


def Extract(hi, lo, a):
    return _op("extract", BitVecSort(hi - lo + 1), a, params=(hi, lo))


def ZeroExt(k, a):
    return _op("zero_extend", BitVecSort(a.size() + k), a, params=(k,))


def SignExt(k, a):
    return _op("sign_extend", BitVecSort(a.size() + k), a, params=(k,))


def Distinct(*a): return _op("distinct", BOOL, *a)
def If(c, a, b): return _op("if", a.sort(), c, a, b)
def And(*a): return _op("and", BOOL, *a)
def Or(*a): return _op("or", BOOL, *a)
def Xor(a, b): return _op("xor", BOOL, a, b)
def Not(a): return _op("not", BOOL, a)
def Implies(a, b): return _op("=>", BOOL, a, b)


def BVMulNoOverflow(a, b, signed):
    assert not signed
    return _op("bvumul_noovfl", BOOL, a, b)


def interpreted(name, sort, *args, params=()):
    """An application by z3's internal name (e.g. ``bvudiv_i``)."""
    return _op(name, sort, *args, params=params)


# -- predicates -----------------------------------------------------------------
def is_app(e): return isinstance(e, Expr)
def is_bv_value(e): return e._value is not None
def is_true(e): return e.decl().name() == "true" and not e._args
def is_false(e): return e.decl().name() == "false" and not e._args
def is_const(e): return not e._args
def is_bv_sort(s): return s.kind == "bv"
def is_bool(e): return e.sort().kind == "bool"
def is_array_sort(s): return s.kind == "array"
def is_K(e): return e.decl().name() == "const" and bool(e._args)


def _ground(e) -> bool:
    seen, stack = set(), [e]
    while stack:
        x = stack.pop()
        if x.get_id() in seen:
            continue
        seen.add(x.get_id())
        if x.decl().kind() == Z3_OP_UNINTERPRETED:
            return False
        stack.extend(x._args)
    return True


def substitute(e, *pairs):
    rep = {a.get_id(): b for a, b in pairs}
    memo = {}

    def go(x):
        if x.get_id() in rep:
            return rep[x.get_id()]
        if x.get_id() in memo:
            return memo[x.get_id()]
        new = [go(a) for a in x._args]
        r = x if all(n is a for n, a in zip(new, x._args)) else _mk(x._decl, new, x._sort, x._value)
        memo[x.get_id()] = r
        return r
    return go(e)


def simplify(e):
    """Ground terms are evaluated (SMT-LIB semantics, via the oracle)."""
    if not _ground(e):
        return e
    from mythril_amd import z3bridge
    from oracle import smtlib_ref as R
    v = R.evaluate([z3bridge.to_node(e, {})], R.Assignment())[0]
    return BoolVal(bool(v)) if e.sort().kind == "bool" else BitVecVal(v, e.size())


class Solver:
    """Decides a query all of whose free constants are pinned by
    ``const == value`` (the check verify() issues)."""

    def __init__(self):
        self.cs: List[Expr] = []
        self.timeout = None

    def set(self, **kw):
        self.timeout = kw.get("timeout")

    def add(self, *cs):
        self.cs.extend(cs)

    def check(self):
        pins: List[Tuple[Expr, Expr]] = []
        for c in self.cs:
            if c.decl().name() == "=" and c._args[0].decl().kind() == Z3_OP_UNINTERPRETED and \
                    not c._args[0]._args:
                pins.append((c._args[0], c._args[1]))
        self._pins = pins
        pin_ids = set()
        for c in self.cs:
            if c.decl().name() == "=" and any(c._args[0] is a for a, _ in pins):
                pin_ids.add(c.get_id())
        cs = [substitute(c, *pins) for c in self.cs if c.get_id() not in pin_ids]
        funs = {}
        for c in cs:                                   # f(k) == v pins of functions
            a = c._args[0] if c._args else None
            if c.decl().name() == "=" and a is not None and a._args and \
                    a.decl().kind() == Z3_OP_UNINTERPRETED and is_bv_value(a._args[0]):
                funs.setdefault(a.decl().name(), []).append((a._args[0], c._args[1]))
        g = And(*cs)
        if funs:
            from mythril_amd import z3bridge
            from mythril_amd.assign import Assignment
            tab = {n: ([(k.as_long(), v.as_long()) for k, v in kv], 0) for n, kv in funs.items()}
            g = z3bridge._replace_ufs(__import__(__name__), g, {n: None for n in funs},
                                      Assignment(funcs=tab))
        r = simplify(g)
        return sat if is_true(r) else (unsat if is_false(r) else unknown)

    def model(self):
        return {a.decl().name(): b for a, b in self._pins}
