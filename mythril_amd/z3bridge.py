"""z3 <-> DAG bridge, used only when z3 is importable (it is not installed in
this image; every function raises :class:`Z3Unavailable` without it).

* :func:`to_node` flattens a z3 AST (what ``laser.smt`` objects hold in
  ``.raw``) into the hash-consed DAG of :mod:`mythril_amd.smt.node`, keyed on
  ``decl().name()`` and deduplicated by ``get_id()``.
  Unknown declarations raise :class:`mythril_amd.ir.Unsupported` → the caller
  falls back to z3.
* :func:`to_z3` rebuilds a z3 expression from a DAG (stock-solver fallback for
  constraints built with the z3-free mirror).
* :func:`verify` substitutes a witness into z3 constraints and simplifies
  (``substitute`` + ``simplify`` must give ``True``), then returns a genuine z3
  model by checking the constraints with the witness as equalities.
"""

from __future__ import annotations

from typing import Dict, List

from .ir import Unsupported
from .smt import node as N


class Z3Unavailable(RuntimeError):
    pass


def _z3():
    try:
        import z3  # noqa: F401
    except ImportError as e:  # pragma: no cover - z3 absent in this image
        raise Z3Unavailable("z3 is not installed") from e
    return z3


def available() -> bool:
    try:
        _z3()
        return True
    except Z3Unavailable:
        return False


_BIN = {"bvadd", "bvsub", "bvmul", "bvudiv", "bvsdiv", "bvurem", "bvsrem", "bvsmod", "bvand",
        "bvor", "bvxor", "bvshl", "bvlshr", "bvashr"}
_CMP = {"bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle", "bvsgt", "bvsge",
        "bvumul_noovfl"}
# z3 internal names of the interpreted division variants (rewriter output)
_DIVI = {"bvudiv_i": "bvudiv", "bvsdiv_i": "bvsdiv", "bvurem_i": "bvurem", "bvsrem_i": "bvsrem",
         "bvsmod_i": "bvsmod"}


def to_node(e, memo: Dict[int, N.Node] = None) -> N.Node:
    z3 = _z3()
    memo = {} if memo is None else memo
    stack = [(e, False)]
    while stack:
        x, done = stack.pop()
        xid = x.get_id()
        if xid in memo:
            continue
        kids = x.children()
        if not done:
            stack.append((x, True))
            stack.extend((k, False) for k in kids if k.get_id() not in memo)
            continue
        a = [memo[k.get_id()] for k in kids]
        name = x.decl().name() if z3.is_app(x) else ""
        name = _DIVI.get(name, name)
        if z3.is_bv_value(x):
            n = N.bv_num(x.as_long(), x.size())
        elif z3.is_true(x):
            n = N.bool_val(True)
        elif z3.is_false(x):
            n = N.bool_val(False)
        elif z3.is_const(x) and x.decl().kind() == z3.Z3_OP_UNINTERPRETED:
            s = x.sort()
            if z3.is_bv_sort(s):
                n = N.bv_var(name, s.size())
            elif z3.is_bool(x):
                n = N.bool_var(name)
            elif z3.is_array_sort(s):
                n = N.array_var(name, s.domain().size(), s.range().size())
            else:
                raise Unsupported("sort %s" % s)
        elif name in _BIN:
            n = N.bv_op(name, *a) if len(a) > 1 else a[0]
        elif name in ("bvneg", "bvnot"):
            n = N.bv_op(name, a[0])
        elif name in _CMP:
            n = N.bv_cmp(name, a[0], a[1])
        elif name == "=":
            n = N.eq(a[0], a[1])
        elif name == "distinct":
            n = N.distinct(*a)
        elif name == "if":
            n = N.ite(a[0], a[1], a[2])
        elif name in ("and", "or", "not", "xor", "=>"):
            n = N.bool_op(name, *a)
        elif name == "concat":
            n = N.concat(*a)
        elif name == "extract":
            hi, lo = x.params()
            n = N.extract(hi, lo, a[0])
        elif name == "zero_extend":
            n = N.zero_extend(x.params()[0], a[0])
        elif name == "sign_extend":
            n = N.sign_extend(x.params()[0], a[0])
        elif name == "select":
            n = N.select(a[0], a[1])
        elif name == "store":
            n = N.store(a[0], a[1], a[2])
        elif name == "const" and z3.is_K(x):
            n = N.const_array(x.sort().domain().size(), a[0])
        elif z3.is_app(x) and x.decl().kind() == z3.Z3_OP_UNINTERPRETED and len(a) == 1:
            n = N.apply_uf(name, kids[0].size(), x.size(), a[0])
        else:
            raise Unsupported("z3 declaration %r" % name)
        memo[xid] = n
    return memo[e.get_id()]


def to_z3(n: N.Node, memo: Dict[int, object] = None):
    z3 = _z3()
    memo = {} if memo is None else memo
    for m in N.topo_order([n]):
        if m.id in memo:
            continue
        a = [memo[x.id] for x in m.args]
        op = m.op
        if op == "bvnum":
            r = z3.BitVecVal(m.params[0], m.width)
        elif op in ("true", "false"):
            r = z3.BoolVal(op == "true")
        elif op == "var":
            r = z3.Bool(m.params[0]) if m.is_bool() else z3.BitVec(m.params[0], m.width)
        elif op == "array":
            r = z3.Array(m.params[0], z3.BitVecSort(m.dom), z3.BitVecSort(m.width))
        elif op == "K":
            r = z3.K(z3.BitVecSort(m.dom), a[0])
        elif op == "store":
            r = z3.Store(a[0], a[1], a[2])
        elif op == "select":
            r = z3.Select(a[0], a[1])
        elif op == "apply":
            f = z3.Function(m.params[0], z3.BitVecSort(m.params[1]), z3.BitVecSort(m.width))
            r = f(a[0])
        elif op in ("bvadd", "bvmul", "bvand", "bvor", "bvxor"):
            fn = {"bvadd": lambda p, q: p + q, "bvmul": lambda p, q: p * q,
                  "bvand": lambda p, q: p & q, "bvor": lambda p, q: p | q,
                  "bvxor": lambda p, q: p ^ q}[op]
            r = a[0]
            for t in a[1:]:
                r = fn(r, t)
        elif op == "bvsub":
            r = a[0] - a[1]
        elif op == "bvneg":
            r = -a[0]
        elif op == "bvnot":
            r = ~a[0]
        elif op == "bvudiv":
            r = z3.UDiv(a[0], a[1])
        elif op == "bvsdiv":
            r = a[0] / a[1]
        elif op == "bvurem":
            r = z3.URem(a[0], a[1])
        elif op == "bvsrem":
            r = z3.SRem(a[0], a[1])
        elif op == "bvsmod":
            r = a[0] % a[1]
        elif op == "bvshl":
            r = a[0] << a[1]
        elif op == "bvlshr":
            r = z3.LShR(a[0], a[1])
        elif op == "bvashr":
            r = a[0] >> a[1]
        elif op == "concat":
            r = z3.Concat(*a)
        elif op == "extract":
            r = z3.Extract(m.params[0], m.params[1], a[0])
        elif op == "zero_extend":
            r = z3.ZeroExt(m.params[0], a[0])
        elif op == "sign_extend":
            r = z3.SignExt(m.params[0], a[0])
        elif op == "=":
            r = a[0] == a[1]
        elif op == "distinct":
            r = z3.Distinct(*a)
        elif op == "ite":
            r = z3.If(a[0], a[1], a[2])
        elif op == "and":
            r = z3.And(*a)
        elif op == "or":
            r = z3.Or(*a)
        elif op == "xor":
            r = z3.Xor(a[0], a[1])
        elif op == "not":
            r = z3.Not(a[0])
        elif op == "=>":
            r = z3.Implies(a[0], a[1])
        elif op in ("bvult", "bvule", "bvugt", "bvuge"):
            r = {"bvult": z3.ULT, "bvule": z3.ULE, "bvugt": z3.UGT, "bvuge": z3.UGE}[op](a[0], a[1])
        elif op in ("bvslt", "bvsle", "bvsgt", "bvsge"):
            r = {"bvslt": lambda p, q: p < q, "bvsle": lambda p, q: p <= q,
                 "bvsgt": lambda p, q: p > q, "bvsge": lambda p, q: p >= q}[op](a[0], a[1])
        elif op == "bvumul_noovfl":
            r = z3.BVMulNoOverflow(a[0], a[1], False)
        else:
            raise Unsupported(op)
        memo[m.id] = r
    return memo[n.id]


def witness_terms(assignment, z3_consts: List[object]):
    """(z3 const, z3 value) pairs for the BV/Bool variables of a witness."""
    z3 = _z3()
    out = []
    for c in z3_consts:
        name = c.decl().name()
        if name in assignment.vars:
            v = assignment.vars[name]
            out.append((c, z3.BoolVal(bool(v)) if z3.is_bool(c) else z3.BitVecVal(v, c.size())))
    return out


def verify(z3_constraints, assignment, timeout_ms: int):
    """Re-verify a GPU witness with z3 and return a z3 model, or None."""
    z3 = _z3()
    consts = set()
    for c in z3_constraints:
        stack = [c]
        while stack:
            x = stack.pop()
            if z3.is_const(x) and x.decl().kind() == z3.Z3_OP_UNINTERPRETED:
                consts.add(x)
            stack.extend(x.children())
    s = z3.Solver()
    s.set(timeout=max(1, int(timeout_ms)))
    s.add(*z3_constraints)
    for c, v in witness_terms(assignment, list(consts)):
        s.add(c == v)
    if s.check() == z3.sat:
        return s.model()
    return None
