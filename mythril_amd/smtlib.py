"""SMT-LIB 2 text for ``get_model`` queries: dump (shared sub-terms named by
``define-fun``) and parse back into the hash-consed DAG
(:mod:`mythril_amd.smt.node`).

Used by the capture / replay tools (:mod:`mythril_amd.capture`, SURVEY.md §8f
rank 2): a query captured on a machine with Mythril + z3 (``Solver.sexpr()``
text) or dumped from DAG nodes here is replayed on the GPU engine.  The parser
accepts the subset z3 prints for the operator vocabulary of SURVEY.md §8a:

* commands ``declare-fun`` / ``declare-const`` / 0-ary ``define-fun`` /
  ``assert`` (others ignored);
* ``let`` bindings (z3's ``a!1``-style sharing), ``|quoted|`` symbols;
* numerals ``(_ bvN w)``, ``#x…``, ``#b…``, ``true`` / ``false``;
* indexed ``(_ extract h l)``, ``(_ zero_extend k)``, ``(_ sign_extend k)``;
* ``((as const (Array (_ BitVec d) (_ BitVec r))) v)``, ``select``, ``store``;
* uninterpreted function applications of declared 1-argument functions;
* z3's internal ``bvudiv_i`` … ``bvsmod_i`` (the same total functions).
"""

from __future__ import annotations

import re
from typing import Dict, List, Optional, Sequence, Tuple

from .smt import node as N

_DIVI = {"bvudiv_i": "bvudiv", "bvsdiv_i": "bvsdiv", "bvurem_i": "bvurem",
         "bvsrem_i": "bvsrem", "bvsmod_i": "bvsmod"}
_BOOL_OPS = {"and", "or", "xor", "not", "=>"}


class ParseError(ValueError):
    pass


# ---------------------------------------------------------------------------
# dump
# ---------------------------------------------------------------------------

def _declarations(roots: Sequence[N.Node]) -> List[str]:
    out, seen = [], set()
    for n in N.topo_order(list(roots)):
        if n.op in ("var", "array"):
            key = ("s", n.params[0])
            if key not in seen:
                seen.add(key)
                out.append("(declare-fun %s () %s)" % (N._quote(n.params[0]), N.sort_sexpr(n)))
        elif n.op == "apply":
            key = ("f", n.params[0])
            if key not in seen:
                seen.add(key)
                out.append("(declare-fun %s ((_ BitVec %d)) (_ BitVec %d))"
                           % (N._quote(n.params[0]), n.params[1], n.width))
    return out


def _head(n: N.Node) -> str:
    if n.op == "extract":
        return "(_ extract %d %d)" % n.params
    if n.op in ("zero_extend", "sign_extend"):
        return "(_ %s %d)" % (n.op, n.params[0])
    if n.op == "apply":
        return N._quote(n.params[0])
    return n.op


def dump_query(constraints: Sequence[N.Node]) -> str:
    """SMT-LIB 2 script with one ``assert`` per constraint; sub-terms used
    more than once are named once with ``define-fun`` (topological order), so
    the text stays linear in the DAG size and parses back to the same
    constraints (:func:`parse_query`)."""
    roots = list(constraints)
    order = N.topo_order(roots)
    uses: Dict[int, int] = {}
    for n in order:
        for a in n.args:
            uses[a.id] = uses.get(a.id, 0) + 1
    leaf_ops = ("bvnum", "true", "false", "var", "array")
    names: Dict[int, str] = {}

    def term(n: N.Node) -> str:
        nm = names.get(n.id)
        if nm is not None:
            return nm
        if n.op == "bvnum":
            return "(_ bv%d %d)" % (n.params[0], n.width)
        if n.op in ("true", "false"):
            return n.op
        if n.op in ("var", "array"):
            return N._quote(n.params[0])
        if n.op == "K":
            return "((as const (Array (_ BitVec %d) (_ BitVec %d))) %s)" % (
                n.dom, n.width, term(n.args[0]))
        return "(" + " ".join([_head(n)] + [term(a) for a in n.args]) + ")"

    lines = ["(set-logic QF_AUFBV)"] + _declarations(roots)
    k = 0
    for n in order:
        if uses.get(n.id, 0) > 1 and n.op not in leaf_ops:
            k += 1
            lines.append("(define-fun a!%d () %s %s)" % (k, N.sort_sexpr(n), term(n)))
            names[n.id] = "a!%d" % k
    lines += ["(assert %s)" % term(c) for c in roots]
    lines.append("(check-sat)")
    return "\n".join(lines) + "\n"


# ---------------------------------------------------------------------------
# parse
# ---------------------------------------------------------------------------

_TOKEN = re.compile(r"\s*(?:;[^\n]*\n?\s*)*(\(|\)|\|[^|]*\||[^\s()|;]+)")


def _tokens(text: str) -> List[str]:
    out, pos = [], 0
    while True:
        m = _TOKEN.match(text, pos)
        if not m:
            break
        out.append(m.group(1))
        pos = m.end()
    if text[pos:].strip():
        raise ParseError("unexpected text at %d" % pos)
    return out


def _sexprs(tokens: List[str]) -> list:
    stack: list = [[]]
    for t in tokens:
        if t == "(":
            stack.append([])
        elif t == ")":
            if len(stack) == 1:
                raise ParseError("unbalanced ')'")
            done = stack.pop()
            stack[-1].append(done)
        else:
            stack[-1].append(t)
    if len(stack) != 1:
        raise ParseError("unbalanced '('")
    return stack[0]


def _sym(t: str) -> str:
    return t[1:-1] if t.startswith("|") and t.endswith("|") else t


def _sort(s) -> Tuple[str, int, int]:
    """(sort, width, dom) of a sort expression."""
    if s == "Bool":
        return N.BOOL, 1, 0
    if isinstance(s, list) and s[:2] == ["_", "BitVec"]:
        return N.BV, int(s[2]), 0
    if isinstance(s, list) and s and s[0] == "Array":
        _, d, _ = _sort(s[1])
        _, r, _ = _sort(s[2])
        return N.ARRAY, r, d
    raise ParseError("unsupported sort %r" % (s,))


class _Env:
    def __init__(self):
        self.consts: Dict[str, N.Node] = {}
        self.funs: Dict[str, Tuple[int, int]] = {}


def _numeral(t: str) -> Optional[N.Node]:
    if t.startswith("#x"):
        return N.bv_num(int(t[2:], 16), 4 * (len(t) - 2))
    if t.startswith("#b"):
        return N.bv_num(int(t[2:], 2), len(t) - 2)
    if t == "true":
        return N.bool_val(True)
    if t == "false":
        return N.bool_val(False)
    return None


def _term(e, env: _Env, scope: Dict[str, N.Node]) -> N.Node:
    if isinstance(e, str):
        n = _numeral(e)
        if n is not None:
            return n
        name = _sym(e)
        if name in scope:
            return scope[name]
        if name in env.consts:
            return env.consts[name]
        raise ParseError("unknown symbol %s" % name)
    if not e:
        raise ParseError("empty term")
    head = e[0]
    if head == "let":
        inner = dict(scope)
        for b in e[1]:
            inner[_sym(b[0])] = _term(b[1], env, scope)    # parallel let
        return _term(e[2], env, inner)
    if isinstance(head, list):
        if head[:1] == ["_"] and head[1].startswith("bv") and head[1][2:].isdigit():
            raise ParseError("numeral applied as a function")
        if head[:1] == ["_"]:
            return _indexed(head, [_term(a, env, scope) for a in e[1:]])
        if head[:1] == ["as"] and head[1] == "const":
            st, w, d = _sort(head[2])
            return N.const_array(d, _term(e[1], env, scope))
        raise ParseError("unsupported head %r" % (head,))
    if head == "_":                                   # (_ bvN w) numeral
        if len(e) == 3 and e[1].startswith("bv"):
            return N.bv_num(int(e[1][2:]), int(e[2]))
        raise ParseError("unsupported indexed term %r" % (e,))
    args = [_term(a, env, scope) for a in e[1:]]
    op = _DIVI.get(head, head)
    name = _sym(head)
    if name in env.funs:
        dom, rng = env.funs[name]
        return N.apply_uf(name, dom, rng, args[0])
    if op in _BOOL_OPS:
        return N.bool_op(op, *args)
    if op == "=":
        return N.eq(*args) if len(args) == 2 else N.bool_op(
            "and", *[N.eq(args[i], args[i + 1]) for i in range(len(args) - 1)])
    if op == "distinct":
        return N.distinct(*args)
    if op == "ite":
        return N.ite(*args)
    if op == "concat":
        return N.concat(*args)
    if op == "select":
        return N.select(*args)
    if op == "store":
        return N.store(*args)
    if op in N._BV_CMP:
        return N.bv_cmp(op, *args)
    if op.startswith("bv"):
        if op in N._BV_NARY and len(args) > 2:
            acc = args[0]
            for a in args[1:]:
                acc = N.bv_op(op, acc, a)
            return acc
        return N.bv_op(op, *args)
    raise ParseError("unsupported operator %s" % op)


def _indexed(head: list, args: List[N.Node]) -> N.Node:
    kind = head[1]
    if kind == "extract":
        return N.extract(int(head[2]), int(head[3]), args[0])
    if kind == "zero_extend":
        return N.zero_extend(int(head[2]), args[0])
    if kind == "sign_extend":
        return N.sign_extend(int(head[2]), args[0])
    raise ParseError("unsupported indexed operator %s" % kind)


def parse_query(text: str) -> List[N.Node]:
    """The asserted constraints of an SMT-LIB 2 script, as DAG nodes, one per
    ``assert``."""
    env = _Env()
    out: List[N.Node] = []
    for cmd in _sexprs(_tokens(text)):
        if not isinstance(cmd, list) or not cmd:
            continue
        c = cmd[0]
        if c == "declare-fun" or c == "declare-const":
            name = _sym(cmd[1])
            if c == "declare-fun" and cmd[2]:
                if len(cmd[2]) != 1:
                    raise ParseError("only 1-argument functions are supported")
                _, dom, _ = _sort(cmd[2][0])
                _, rng, _ = _sort(cmd[3])
                env.funs[name] = (dom, rng)
                continue
            st, w, d = _sort(cmd[3] if c == "declare-fun" else cmd[2])
            if st == N.BOOL:
                env.consts[name] = N.bool_var(name)
            elif st == N.BV:
                env.consts[name] = N.bv_var(name, w)
            else:
                env.consts[name] = N.array_var(name, d, w)
        elif c == "define-fun":
            if cmd[2]:
                raise ParseError("define-fun with parameters is not supported")
            env.consts[_sym(cmd[1])] = _term(cmd[4], env, {})
        elif c == "assert":
            out.append(_term(cmd[1], env, {}))
    return out
