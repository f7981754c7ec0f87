"""ABI layout presets for the witness search (search mode only).

LASER reads a dynamic parameter (``batchTransfer(address[] _receivers, ...)``)
at ``calldata[off + 4 + i]`` where ``off`` is itself the calldata word at byte
4 + 32k (``calldata.py:207-232``: a symbolic offset gives the index
``off + i``).  A search that guesses ``off`` reads the array at a random
offset — and in the compiled program every such read is a lookup compared
with every other calldata key.  z3 picks ``off``; the search does what the
Solidity ABI does: the dynamic data of a call starts right after its head,
32-aligned, in parameter order.

:func:`plan` finds, per calldata array, the offset words its symbolic reads
are based on and pins them (and ``calldatasize``) to that layout: the offset
words' bytes and the size become **presets** — fixed parts of every
candidate model — and the query is rewritten with them substituted (the
offset bytes become numerals, every read key ``off + c`` the numeral
``K + c``), so every read is a constant-key read.  The rewritten query is
the original one evaluated under the presets, and :func:`merge` adds the
presets to a witness, so a witness is a model of the ORIGINAL query (its
checks — the oracle in the tests, z3 in production — see the preset values).
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from .smt import node as N
from .smt.node import Node, topo_order


class View:
    """A node of the query under the presets (:meth:`Plan.view`): the same
    fields as ``smt.node.Node``, its id that of the node it stands for."""
    __slots__ = ("op", "sort", "width", "dom", "args", "params", "id")

    def __init__(self, op, sort, width, dom, args, params, nid):
        self.op, self.sort, self.width, self.dom = op, sort, width, dom
        self.args, self.params, self.id = args, params, nid

    def is_bool(self) -> bool:
        return self.sort == N.BOOL

    def is_bv(self) -> bool:
        return self.sort == N.BV

    def is_array(self) -> bool:
        return self.sort == N.ARRAY


@dataclass
class Plan:
    vars: Dict[str, int] = field(default_factory=dict)             # calldatasize
    arrays: Dict[str, Dict[int, int]] = field(default_factory=dict)  # offset bytes
    subst: Dict[int, int] = field(default_factory=dict)            # node id -> numeral value

    def apply(self, nodes: Sequence[Node]) -> List[Node]:
        """``nodes`` with the preset cells, the size and the pinned read
        keys replaced by numerals (hash-consed rebuild, linear)."""
        memo: Dict[int, Node] = {}
        for n in topo_order(list(nodes)):
            v = self.subst.get(n.id)
            if v is not None:
                r = N.bv_num(v, n.width)
            else:
                args = tuple(memo[a.id] for a in n.args)
                r = n if all(a is b for a, b in zip(args, n.args)) else \
                    N.mk(n.op, n.sort, n.width, args, n.params, dom=n.dom)
            memo[n.id] = r
        return [memo[n.id] for n in nodes]

    def view(self, nodes: Sequence[Node]) -> List[object]:
        """The query the search compiles (``ir.compile_constraints`` with
        ``abi_presets``): like :meth:`apply`, but every replaced node keeps
        the id of the node it replaces and nothing is hash-consed — so the
        program's schedule (ordered by source ids) follows the original
        query, and the native compiler (include/mythcc.h), which substitutes
        in place, builds the same program."""
        memo: Dict[int, object] = {}
        for n in topo_order(list(nodes)):
            v = self.subst.get(n.id)
            if v is not None:
                r = View("bvnum", N.BV, n.width, 0, (), (v % (1 << n.width),), n.id)
            else:
                args = tuple(memo[a.id] for a in n.args)
                r = n if all(a is b for a, b in zip(args, n.args)) else \
                    View(n.op, n.sort, n.width, n.dom, args, n.params, n.id)
            memo[n.id] = r
        return [memo[n.id] for n in nodes]


def _split_add(k: Node) -> Tuple[Optional[Node], int]:
    """``k`` as base + constant (bvadd chains with numerals)."""
    c, base, stack = 0, None, [k]
    while stack:
        x = stack.pop()
        if x.op == "bvnum":
            c += x.params[0]
        elif x.op == "bvadd":
            stack.extend(x.args)
        elif base is None:
            base = x
        else:
            return None, 0
    return base, c % (1 << k.width)


def _byte_cell(x: Node, arr: Node) -> Tuple[Optional[int], Optional[Node]]:
    """(offset, size var) of one calldata byte ``ite(p < size, A[p], 0)`` or
    ``A[p]`` with a numeral p."""
    size = None
    if x.op == "ite" and x.args[2].op == "bvnum" and x.args[2].params[0] == 0:
        c = x.args[0]
        if c.op != "bvslt" or c.args[0].op != "bvnum" or c.args[1].op != "var":
            return None, None
        size = c.args[1]
        x = x.args[1]
    if x.op == "select" and x.args[0] is arr and x.args[1].op == "bvnum":
        return x.args[1].params[0], size
    return None, None


def _word(base: Node, arr: Node) -> Tuple[Optional[int], Optional[Node]]:
    """(first byte offset, size var) when ``base`` is the 32-byte word of
    ``arr`` at a constant offset."""
    parts, stack = [], [base]
    while stack:
        x = stack.pop()
        if x.op == "concat":
            stack.extend(reversed(x.args))
        else:
            parts.append(x)
    if len(parts) != 32:
        return None, None
    offs, size = [], None
    for p in parts:
        o, s = _byte_cell(p, arr)
        if o is None or (s is not None and size is not None and s is not size):
            return None, None
        size = s or size
        offs.append(o)
    if offs != list(range(offs[0], offs[0] + 32)):
        return None, None
    return offs[0], size


def plan(constraints: Sequence[Node]) -> Optional[Plan]:
    nodes = topo_order(list(constraints))
    by_arr: Dict[int, dict] = {}
    for n in nodes:
        if n.op != "select" or n.args[0].op != "array":
            continue
        arr, k = n.args
        d = by_arr.setdefault(arr.id, {"arr": arr, "const": set(), "sym": []})
        if k.op == "bvnum":
            d["const"].add(k.params[0])
        else:
            d["sym"].append(k)
    out = Plan()
    for d in by_arr.values():
        arr = d["arr"]
        if not d["sym"] or not d["const"]:
            continue
        bases: Dict[int, list] = {}           # base id -> [base, lo c, hi c, offset, keys]
        ok = True
        for k in d["sym"]:
            base, c = _split_add(k)
            if base is None or c >> 32:
                ok = False
                break
            r = bases.get(base.id)
            if r is None:
                off, size = _word(base, arr)
                if off is None:
                    ok = False
                    break
                r = bases[base.id] = [base, c, c, off, [], size]
            r[1], r[2] = min(r[1], c), max(r[2], c)
            r[4].append((k, c))
        if not ok:
            continue
        size_var = None
        nxt = max(d["const"]) + 1
        cells: Dict[int, int] = {}
        for base, lo, hi, off, keys, size in bases.values():
            # the read at base + lo lands 32-aligned past everything read so far
            val = -(-(nxt - lo) // 32) * 32
            for i in range(32):
                cells[off + i] = (val >> (8 * (31 - i))) & 0xFF
            for k, c in keys:
                out.subst[k.id] = (val + c) % (1 << k.width)
            nxt = val + hi + 1
            size_var = size_var or size
        if size_var is not None:
            out.vars[size_var.params[0]] = nxt
            out.subst[size_var.id] = nxt % (1 << size_var.width)
        out.arrays[arr.params[0]] = cells
        for n in nodes:
            if n.op == "select" and n.args[0] is arr and n.args[1].op == "bvnum" and \
                    n.args[1].params[0] in cells:
                out.subst[n.id] = cells[n.args[1].params[0]] % (1 << n.width)
    return out if out.arrays else None


def merge(asg, presets: Optional[Plan]):
    """A witness of the rewritten query + the presets = a model of the
    original query (preset cells first in their tables: first-match)."""
    if presets is None:
        return asg
    for name, v in presets.vars.items():
        asg.vars[name] = v
    for name, cells in presets.arrays.items():
        entries, default = asg.arrays.get(name, ([], 0))
        asg.arrays[name] = ([(k, v) for k, v in sorted(cells.items())] +
                            [e for e in entries if e[0] not in cells], default)
    return asg
