"""Candidate assignments (models) and their SoA packing for the engine.

An assignment interprets every free symbol of a constraint set the way a z3
model does (``mythril/laser/smt/model.py``): bit-vector / Bool variables get a
value, free arrays and uninterpreted functions get a finite table of
``(key -> value)`` entries (first match wins) plus an ``else`` value.
"""

from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

from .ir import CHUNK, Program

Table = Tuple[List[Tuple[int, int]], int]


class Assignment:
    def __init__(self, vars: Dict[str, int] = None, arrays: Dict[str, Table] = None,
                 funcs: Dict[str, Table] = None):
        self.vars = dict(vars or {})
        self.arrays = dict(arrays or {})
        self.funcs = dict(funcs or {})

    def table(self, name: str) -> Table:
        if name in self.arrays:
            return self.arrays[name]
        if name in self.funcs:
            return self.funcs[name]
        return ([], 0)

    def __repr__(self):
        return "Assignment(vars=%r, arrays=%r, funcs=%r)" % (self.vars, self.arrays, self.funcs)


def _padded_entries(tab: Table, n: int) -> List[Tuple[int, int]]:
    entries, default = tab
    if len(entries) > n:
        raise ValueError("table has %d entries, program was compiled for %d" % (len(entries), n))
    entries = list(entries)
    filler = entries[0] if entries else (0, default)
    return entries + [filler] * (n - len(entries))


def lookup(tab: Table, key: int) -> int:
    """First-match table semantics (how a z3 model interprets an array)."""
    entries, default = tab
    for k, v in entries:
        if k == key:
            return v
    return default


def leaf_values(program: Program, asg: Assignment) -> List[int]:
    out = []
    for leaf in program.leaves:
        if leaf.kind == "var":
            v = asg.vars.get(leaf.source, 0)
        elif leaf.kind == "aux":          # search-mode selector: not part of a model
            v = 0
        else:
            tab = asg.table(leaf.source)
            if leaf.kind == "cval":
                v = lookup(tab, program.table_ckeys[leaf.source][leaf.entry])
            elif leaf.kind == "else":
                v = tab[1]
            else:
                # entries at constant keys are served by the cval leaves
                ck = set(program.table_ckeys.get(leaf.source, ()))
                rest = ([e for e in tab[0] if e[0] not in ck], tab[1]) if ck else tab
                ent = _padded_entries(rest, program.table_sizes[leaf.source])[leaf.entry]
                v = ent[0] if leaf.kind == "key" else ent[1]
        v = int(v) >> (CHUNK * leaf.chunk)
        out.append(v & ((1 << leaf.width) - 1))
    return out


def pack(program: Program, assignments: Sequence[Assignment]) -> np.ndarray:
    """(n_leaves, 8, n) uint32 little-endian limbs."""
    n = len(assignments)
    out = np.zeros((len(program.leaves), 8, n), dtype=np.uint32)
    for a, asg in enumerate(assignments):
        for i, v in enumerate(leaf_values(program, asg)):
            for j in range(8):
                out[i, j, a] = (v >> (32 * j)) & 0xFFFFFFFF
    return out


def _limbs_int(row) -> int:
    return int.from_bytes(np.ascontiguousarray(row, dtype="<u4").tobytes(), "little")


def _rows_int(rows: np.ndarray, n: int) -> list:
    """The first n rows of an (.., 8) limb array as Python ints (one byte
    string, sliced: no per-limb Python work)."""
    b = np.ascontiguousarray(rows[:n], dtype="<u4").tobytes()
    return [int.from_bytes(b[32 * i:32 * i + 32], "little") for i in range(n)]


def unpack(program: Program, leaves: np.ndarray, probes: np.ndarray = None) -> Assignment:
    """Inverse of :func:`pack` for one candidate: leaves is (n_leaves, 8).  A
    solve-mode program (``Program.solved``) also needs the candidate's probe
    values ((n_probes, 8)): the leaves it defines by equalities and the keys
    of its argument-keyed table entries are computed, not generated."""
    vals = _rows_int(leaves, len(program.leaves))
    pv = _rows_int(probes, len(probes)) if probes is not None else None
    if program.solved:
        if probes is None:
            raise ValueError("a solve-mode witness needs its probe values")
        for li, k in program.derived.items():
            vals[li] = pv[k]
    vars_: Dict[str, int] = {}
    tables: Dict[str, dict] = {}
    for leaf, v in zip(program.leaves, vals):
        part = v << (CHUNK * leaf.chunk)
        if leaf.kind == "aux":
            continue
        if leaf.kind == "var":
            vars_[leaf.source] = vars_.get(leaf.source, 0) | part
        else:
            t = tables.setdefault(leaf.source, {"k": {}, "v": {}, "c": {}, "else": 0})
            if leaf.kind == "cval":
                t["c"][leaf.entry] = t["c"].get(leaf.entry, 0) | part
            elif leaf.kind == "else":
                t["else"] |= part
            else:
                d = t["k" if leaf.kind == "key" else "v"]
                d[leaf.entry] = d.get(leaf.entry, 0) | part
    for name, ents in program.entry_keys.items():
        t = tables.setdefault(name, {"k": {}, "v": {}, "c": {}, "else": 0})
        for e, chunks in enumerate(ents):
            t["k"][e] = sum(pv[k] << (CHUNK * c) for c, k in enumerate(chunks))
    arrays, funcs = {}, {}
    for name, t in tables.items():
        n = program.table_sizes.get(name, 0)
        ck = program.table_ckeys.get(name, [])
        tab = ([(c, t["c"].get(i, 0)) for i, c in enumerate(ck)] +
               [(t["k"].get(e, 0), t["v"].get(e, 0)) for e in range(n)], t["else"])
        (funcs if program.table_kinds.get(name) == "func" else arrays)[name] = tab
    asg = Assignment(vars_, arrays, funcs)
    if getattr(program, "presets", None) is not None:
        from .abi import merge
        merge(asg, program.presets)
    return asg
