"""z3 <-> DAG bridge, used only when z3 is importable (it is not installed in
this image; every function raises :class:`Z3Unavailable` without it).

* :func:`to_node` flattens a z3 AST (what ``laser.smt`` objects hold in
  ``.raw``) into the hash-consed DAG of :mod:`mythril_amd.smt.node`, keyed on
  ``decl().name()`` and deduplicated by ``get_id()``.
  Unknown declarations raise :class:`mythril_amd.ir.Unsupported` → the caller
  falls back to z3.
* :func:`to_z3` rebuilds a z3 expression from a DAG (stock-solver fallback for
  constraints built with the z3-free mirror).
* :func:`verify` substitutes a whole witness into the z3 constraints (BV and
  Bool values, arrays as ``K`` + ``Store`` terms, uninterpreted functions as
  ite chains over their tables), requires ``simplify`` to give ``True``, and
  only then returns a genuine z3 model from a ``Solver`` check with every
  symbol pinned.
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


def _symbols(z3_constraints):
    """Free constants (BV / Bool / array) and uninterpreted function decls of
    the constraints: one visit per hash-consed node (``get_id``), so shared
    sub-terms (calldata words over one ``size``, long store chains) are
    walked once, not once per tree path."""
    z3 = _z3()
    consts, funcs = {}, {}
    seen = set()
    stack = list(z3_constraints)
    while stack:
        x = stack.pop()
        xid = x.get_id()
        if xid in seen:
            continue
        seen.add(xid)
        if z3.is_app(x) and x.decl().kind() == z3.Z3_OP_UNINTERPRETED:
            if z3.is_const(x):
                consts[xid] = x
            else:
                funcs[x.decl().name()] = x.decl()
        stack.extend(x.children())
    return list(consts.values()), funcs


def _table_term(z3, dom_sort, rng_sort, table):
    """A free array's model table as ``Store(...Store(K(dom, else), k, v)...)``,
    first entry outermost (first match wins, as the witness reads it)."""
    entries, default = table
    t = z3.K(dom_sort, z3.BitVecVal(default, rng_sort.size()))
    for k, v in reversed(entries):
        t = z3.Store(t, z3.BitVecVal(k, dom_sort.size()), z3.BitVecVal(v, rng_sort.size()))
    return t


def _uf_term(z3, arg, rng_size, table):
    entries, default = table
    t = z3.BitVecVal(default, rng_size)
    for k, v in reversed(entries):
        t = z3.If(arg == z3.BitVecVal(k, arg.size()), z3.BitVecVal(v, rng_size), t)
    return t


def interpretation(assignment, consts):
    """(z3 const, value term) pairs interpreting every free constant of the
    witness; a symbol the witness does not mention did not influence the
    device evaluation, so any value is consistent: 0 / false / K(0)."""
    z3 = _z3()
    out = []
    for c in consts:
        name = c.decl().name()
        s = c.sort()
        if z3.is_bool(c):
            out.append((c, z3.BoolVal(bool(assignment.vars.get(name, 0)))))
        elif z3.is_bv_sort(s):
            out.append((c, z3.BitVecVal(assignment.vars.get(name, 0), s.size())))
        elif z3.is_array_sort(s):
            out.append((c, _table_term(z3, s.domain(), s.range(),
                                       assignment.arrays.get(name, ([], 0)))))
    return out


def _replace_ufs(z3, e, funcs, assignment):
    """Rebuild ``e`` with every application of an uninterpreted function
    replaced by the ite chain over the witness's table for it."""
    if not funcs:
        return e
    memo: Dict[int, object] = {}
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
        new = [memo[k.get_id()] for k in kids]
        if z3.is_app(x) and x.decl().kind() == z3.Z3_OP_UNINTERPRETED and kids:
            name = x.decl().name()
            r = _uf_term(z3, new[0], x.size(), assignment.funcs.get(name, ([], 0)))
        elif kids and any(n.get_id() != k.get_id() for n, k in zip(new, kids)):
            r = x.decl()(*new)
        else:
            r = x
        memo[xid] = r
    return memo[e.get_id()]


def verify(z3_constraints, assignment, timeout_ms: int):
    """Re-verify a GPU witness with z3: substitute the whole
    witness — BV / Bool values, arrays as ``K`` + ``Store`` terms, UF
    applications as ite chains over their tables — and require ``simplify``
    to give ``True``; only then ask a ``Solver`` (every symbol pinned, so the
    check is immediate) for a genuine z3 model.  None if z3 disagrees."""
    z3 = _z3()
    consts, funcs = _symbols(z3_constraints)
    pins = interpretation(assignment, consts)
    ground = z3.And(*z3_constraints) if len(z3_constraints) != 1 else z3_constraints[0]
    ground = _replace_ufs(z3, z3.substitute(ground, *pins) if pins else ground, funcs, assignment)
    if not z3.is_true(z3.simplify(ground)):
        return None
    s = z3.Solver()
    s.set(timeout=max(1, int(timeout_ms)))
    s.add(*z3_constraints)
    for c, v in pins:
        s.add(c == v)
    for name, f in funcs.items():
        for k, v in assignment.funcs.get(name, ([], 0))[0]:
            s.add(f(z3.BitVecVal(k, f.domain(0).size())) == z3.BitVecVal(v, f.range().size()))
    if s.check() == z3.sat:
        return s.model()
    return None
