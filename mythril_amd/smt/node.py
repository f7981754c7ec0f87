"""Hash-consed expression DAG nodes (the z3 AST stand-in for the drop-in).

The reference builds every constraint as a z3 AST (``mythril/laser/smt/*.py``
wrap ``z3.ExprRef``); z3 hash-conses those ASTs, so equal sub-terms are one
node with one ``get_id()``.  This module gives the same structure without z3:
a ``Node`` is immutable, created only through :func:`mk`, and structurally
equal nodes are the same object.  Operator names are the SMT-LIB 2.6 names z3
reports from ``decl().name()`` so that a z3 front-end and the SMT-LIB parser
produce identical DAGs.

Sorts: ``BV`` (width >= 1), ``BOOL`` and ``ARRAY`` (domain width -> range
width).  Uninterpreted functions are ``apply`` nodes whose params carry the
function name and signature (reference ``mythril/laser/smt/function.py:7-25``).
"""

from __future__ import annotations

import contextlib
import itertools
import threading
from typing import Dict, Tuple

BV = "bv"
BOOL = "bool"
ARRAY = "array"

_ids = itertools.count(1)
_table: Dict[tuple, "Node"] = {}
_lock = threading.Lock()


class Node:
    """One DAG node.  ``width`` is the bit-width for BV, 1 for BOOL and the
    range width for ARRAY (``dom`` holds the domain width)."""

    # _enc: the native compiler's walk record of this node (set on its first
    # walk, csrc/mg_compile_py.cpp encode)
    __slots__ = ("op", "sort", "width", "dom", "args", "params", "id", "_h", "_enc")

    def __init__(self, op, sort, width, dom, args, params):
        self.op = op
        self.sort = sort
        self.width = width
        self.dom = dom
        self.args = args
        self.params = params
        self.id = next(_ids)
        self._h = hash((op, sort, width, dom, tuple(a.id for a in args), params))

    def __hash__(self):
        return self._h

    # identity equality: hash-consing makes structural == identity
    def __eq__(self, other):
        return self is other

    def __ne__(self, other):
        return self is not other

    def is_bool(self) -> bool:
        return self.sort == BOOL

    def is_bv(self) -> bool:
        return self.sort == BV

    def is_array(self) -> bool:
        return self.sort == ARRAY

    def __repr__(self):
        return to_sexpr(self, max_depth=4)


def mk(op: str, sort: str, width: int, args: Tuple[Node, ...] = (), params: tuple = (),
       dom: int = 0) -> Node:
    """Return the unique node for this structure (hash-consing)."""
    key = (op, sort, width, dom, tuple(a.id for a in args), params)
    n = _table.get(key)
    if n is not None:
        return n
    with _lock:
        n = _table.get(key)
        if n is None:
            n = Node(op, sort, width, dom, tuple(args), params)
            _table[key] = n
    return n


def find(op: str, sort: str, width: int, args: Tuple[Node, ...] = (), params: tuple = (),
         dom: int = 0):
    """The node of this structure if it exists, else None (never creates
    one: mythril_amd/refute.py looks up terms other atoms may share)."""
    return _table.get((op, sort, width, dom, tuple(a.id for a in args), params))


@contextlib.contextmanager
def fresh_scope():
    """Build inside an empty hash-consing table (the previous one is restored
    afterwards).  Node ids then follow the construction order of what is
    built inside alone — not which equal nodes this process happened to
    build before — so a compiled program's schedule (ordered by source ids,
    ir._schedule) is the same in every process.  Nodes built inside are not
    shared with equal nodes outside."""
    global _table
    with _lock:
        saved, _table = _table, {}
    try:
        yield
    finally:
        with _lock:
            _table = saved


# ----------------------------------------------------------------------------
# constructors used by the front-ends (laser.smt mirror, SMT-LIB parser, z3)
# ----------------------------------------------------------------------------

def bv_num(value: int, width: int) -> Node:
    if width <= 0:
        raise ValueError("bit-vector width must be positive")
    return mk("bvnum", BV, width, (), (value % (1 << width),))


def bv_var(name: str, width: int) -> Node:
    return mk("var", BV, width, (), (name,))


def bool_val(v: bool) -> Node:
    return mk("true" if v else "false", BOOL, 1)


def bool_var(name: str) -> Node:
    return mk("var", BOOL, 1, (), (name,))


def array_var(name: str, dom: int, rng: int) -> Node:
    return mk("array", ARRAY, rng, (), (name,), dom=dom)


def const_array(dom: int, value: Node) -> Node:
    return mk("K", ARRAY, value.width, (value,), (), dom=dom)


def select(arr: Node, idx: Node) -> Node:
    _check(arr.is_array() and idx.is_bv() and idx.width == arr.dom, "select sort mismatch")
    return mk("select", BV, arr.width, (arr, idx))


def store(arr: Node, idx: Node, val: Node) -> Node:
    _check(arr.is_array() and idx.width == arr.dom and val.width == arr.width,
           "store sort mismatch")
    return mk("store", ARRAY, arr.width, (arr, idx, val), dom=arr.dom)


def apply_uf(fname: str, dom: int, rng: int, arg: Node) -> Node:
    _check(arg.is_bv() and arg.width == dom, "UF argument width mismatch")
    return mk("apply", BV, rng, (arg,), (fname, dom))


_BV_BIN = {"bvadd", "bvsub", "bvmul", "bvudiv", "bvsdiv", "bvurem", "bvsrem", "bvsmod",
           "bvand", "bvor", "bvxor", "bvshl", "bvlshr", "bvashr"}
_BV_NARY = {"bvadd", "bvmul", "bvand", "bvor", "bvxor"}
_BV_CMP = {"bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle", "bvsgt", "bvsge",
           "bvumul_noovfl"}


def bv_op(op: str, *args: Node) -> Node:
    if op in ("bvneg", "bvnot"):
        _check(len(args) == 1 and args[0].is_bv(), op + " arity")
        return mk(op, BV, args[0].width, args)
    _check(op in _BV_BIN, "unknown bit-vector op " + op)
    _check(len(args) >= 2 and (len(args) == 2 or op in _BV_NARY), op + " arity")
    w = args[0].width
    for a in args:
        _check(a.is_bv() and a.width == w, op + " width mismatch")
    return mk(op, BV, w, args)


def bv_cmp(op: str, a: Node, b: Node) -> Node:
    _check(op in _BV_CMP, "unknown comparison " + op)
    _check(a.is_bv() and b.is_bv() and a.width == b.width, op + " width mismatch")
    return mk(op, BOOL, 1, (a, b))


def eq(a: Node, b: Node) -> Node:
    _check(a.sort == b.sort and a.width == b.width and a.dom == b.dom, "= sort mismatch")
    return mk("=", BOOL, 1, (a, b))


def distinct(*args: Node) -> Node:
    return mk("distinct", BOOL, 1, args)


def concat(*args: Node) -> Node:
    _check(len(args) >= 1 and all(a.is_bv() for a in args), "concat sorts")
    if len(args) == 1:
        return args[0]
    return mk("concat", BV, sum(a.width for a in args), args)


def extract(hi: int, lo: int, a: Node) -> Node:
    _check(a.is_bv() and 0 <= lo <= hi < a.width, "extract bounds")
    return mk("extract", BV, hi - lo + 1, (a,), (hi, lo))


def zero_extend(k: int, a: Node) -> Node:
    _check(k >= 0 and a.is_bv(), "zero_extend")
    if k == 0:
        return a
    return mk("zero_extend", BV, a.width + k, (a,), (k,))


def sign_extend(k: int, a: Node) -> Node:
    _check(k >= 0 and a.is_bv(), "sign_extend")
    if k == 0:
        return a
    return mk("sign_extend", BV, a.width + k, (a,), (k,))


def ite(c: Node, a: Node, b: Node) -> Node:
    _check(c.is_bool(), "ite condition must be Bool")
    _check(a.sort == b.sort and a.width == b.width and a.dom == b.dom, "ite branch sorts")
    return mk("ite", a.sort, a.width, (c, a, b), dom=a.dom)


def bool_op(op: str, *args: Node) -> Node:
    _check(op in ("and", "or", "xor", "not", "=>"), "unknown boolean op " + op)
    _check(all(a.is_bool() for a in args), op + " needs Bool arguments")
    if op == "not":
        _check(len(args) == 1, "not arity")
    elif op in ("xor", "=>"):
        _check(len(args) == 2, op + " arity")
    if op in ("and", "or") and len(args) == 1:
        return args[0]
    if op == "and" and not args:
        return bool_val(True)
    if op == "or" and not args:
        return bool_val(False)
    return mk(op, BOOL, 1, args)


class SortError(TypeError):
    pass


def _check(cond: bool, msg: str) -> None:
    if not cond:
        raise SortError(msg)


# ----------------------------------------------------------------------------
# traversal / printing
# ----------------------------------------------------------------------------

def topo_order(roots) -> list:
    """Post-order (children first) list of every node reachable from roots,
    each exactly once.  Iterative, so deep Concat chains do not recurse."""
    seen = set()
    out = []
    for r in roots:
        if r.id in seen:
            continue
        stack = [(r, False)]
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


def sort_sexpr(n: Node) -> str:
    if n.sort == BOOL:
        return "Bool"
    if n.sort == BV:
        return "(_ BitVec %d)" % n.width
    return "(Array (_ BitVec %d) (_ BitVec %d))" % (n.dom, n.width)


def _quote(name: str) -> str:
    if name and all(ch.isalnum() or ch in "_.$@!%^&*-+<>=?/~" for ch in name) \
            and not name[0].isdigit():
        return name
    return "|" + name.replace("|", "") + "|"


def to_sexpr(n: Node, max_depth: int = -1) -> str:
    """SMT-LIB 2 text of one term (no sharing; for debugging — whole queries
    are written by :func:`mythril_amd.smtlib.dump_query`)."""
    if max_depth == 0:
        return "..."
    op = n.op
    if op == "bvnum":
        return "(_ bv%d %d)" % (n.params[0], n.width)
    if op in ("true", "false"):
        return op
    if op in ("var", "array"):
        return _quote(n.params[0])
    sub = [to_sexpr(a, max_depth - 1) for a in n.args]
    if op == "extract":
        head = "(_ extract %d %d)" % n.params
    elif op in ("zero_extend", "sign_extend"):
        head = "(_ %s %d)" % (op, n.params[0])
    elif op == "K":
        return "((as const (Array (_ BitVec %d) (_ BitVec %d))) %s)" % (n.dom, n.width, sub[0])
    elif op == "apply":
        head = _quote(n.params[0])
    else:
        head = op
    return "(" + " ".join([head] + sub) + ")"
