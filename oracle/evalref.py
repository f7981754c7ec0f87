"""ORACLE — test infrastructure / CPU baseline only.

ctypes wrapper of ``oracle/evalref.c`` (the C restatement of z3's evaluation
of a get_model DAG).  :func:`serialize` flattens a SOURCE constraint DAG into
the C oracle's node records; leaves are numbered like the compiled
:class:`mythril_amd.ir.Program` so both sides read the same assignment.
"""

from __future__ import annotations

import ctypes as C
import os
from typing import Dict, List, Sequence

import numpy as np

from mythril_amd.smt.node import Node, topo_order

from . import build as _build

E = {name: i + 1 for i, name in enumerate(
    "NUM VAR TRUE FALSE ADD SUB MUL UDIV UREM SDIV SREM SMOD AND OR XOR NOT NEG SHL LSHR ASHR "
    "CONCAT EXTRACT ZEXT SEXT EQ ULT ULE SLT SLE UMULNO ITE BAND BOR BXOR BNOT SELECT STORE "
    "KARR ARRVAR APPLY".split())}

_BIN = {"bvadd": "ADD", "bvsub": "SUB", "bvmul": "MUL", "bvudiv": "UDIV", "bvurem": "UREM",
        "bvsdiv": "SDIV", "bvsrem": "SREM", "bvsmod": "SMOD", "bvand": "AND", "bvor": "OR",
        "bvxor": "XOR", "bvshl": "SHL", "bvlshr": "LSHR", "bvashr": "ASHR"}
_CMP = {"bvult": ("ULT", 0), "bvule": ("ULE", 0), "bvugt": ("ULT", 1), "bvuge": ("ULE", 1),
        "bvslt": ("SLT", 0), "bvsle": ("SLE", 0), "bvsgt": ("SLT", 1), "bvsge": ("SLE", 1),
        "bvumul_noovfl": ("UMULNO", 0)}


class TableDesc(C.Structure):
    _fields_ = [("key_w", C.c_uint32), ("val_w", C.c_uint32), ("entries", C.c_uint32),
                ("else_leaf", C.c_uint32), ("key_leaf_off", C.c_uint32),
                ("val_leaf_off", C.c_uint32), ("n_ckeys", C.c_uint32),
                ("ckey_off", C.c_uint32), ("cval_leaf_off", C.c_uint32)]


class Serialized:
    def __init__(self):
        self.recs: List[List[int]] = []
        self.consts: List[int] = []
        self.roots: List[int] = []
        self.tables: List[TableDesc] = []
        self.leafidx: List[int] = []
        self.node_index: Dict[int, int] = {}


def serialize(constraints: Sequence[Node], program, probes: Sequence[Node] = ()) -> Serialized:
    li = program.leaf_index()
    S = Serialized()
    const_ix: Dict[int, int] = {}
    table_ix: Dict[str, int] = {}

    def rec(op, w, a0=0, a1=0, a2=0, p0=0, p1=0):
        S.recs.append([E[op], w, a0, a1, a2, p0, p1, 0])
        return len(S.recs) - 1

    def const(v):
        if v not in const_ix:
            const_ix[v] = len(S.consts)
            S.consts.append(v)
        return const_ix[v]

    def table(name, key_w, val_w):
        if name not in table_ix:
            n = program.table_sizes[name]
            koff = len(S.leafidx)
            # leaves of entries a program never consults (a table read only
            # at its constant keys) are absent: index them as leaf 0
            S.leafidx += [li.get("%s#k%d#0" % (name, e), 0) for e in range(n)]
            voff = len(S.leafidx)
            S.leafidx += [li.get("%s#v%d#0" % (name, e), 0) for e in range(n)]
            # constant-keyed entries first (ir.scan_const_keys): key constant
            # indices, then their value leaves (a value leaf a query never
            # reads is absent from the program: index it as leaf 0, which the
            # lookup below then never reaches for a different key)
            ck = program.table_ckeys.get(name, [])
            ckoff = len(S.leafidx)
            S.leafidx += [const(c) for c in ck]
            cvoff = len(S.leafidx)
            S.leafidx += [li.get("%s#c%d#0" % (name, i), 0) for i in range(len(ck))]
            table_ix[name] = len(S.tables)
            S.tables.append(TableDesc(key_w, val_w, n, li.get("%s#else#0" % name, 0), koff, voff,
                                      len(ck), ckoff, cvoff))
        return table_ix[name]

    ix = S.node_index
    for n in topo_order(list(constraints) + list(probes)):
        op, w = n.op, n.width
        a = [ix.get(x.id, 0) for x in n.args]
        if op == "bvnum":
            r = rec("NUM", w, p0=const(n.params[0]))
        elif op == "var":
            name = n.params[0] if w <= 256 else n.params[0] + "#0"
            r = rec("VAR", w, p0=li[name])
        elif op in ("true", "false"):
            r = rec(op.upper(), 1)
        elif op in _BIN:
            r = a[0]
            for x in a[1:]:
                r = rec(_BIN[op], w, r, x)
        elif op in ("bvnot", "not"):
            r = rec("NOT" if op == "bvnot" else "BNOT", w, a[0])
        elif op == "bvneg":
            r = rec("NEG", w, a[0])
        elif op in ("and", "or"):
            r = a[0]
            for x in a[1:]:
                r = rec("BAND" if op == "and" else "BOR", 1, r, x)
        elif op == "xor":
            r = rec("BXOR", 1, a[0], a[1])
        elif op == "=>":
            r = rec("BOR", 1, rec("BNOT", 1, a[0]), a[1])
        elif op in _CMP:
            name, swap = _CMP[op]
            x, y = (a[1], a[0]) if swap else (a[0], a[1])
            r = rec(name, 1, x, y, p0=n.args[0].width)
        elif op == "=":
            r = rec("EQ", 1, a[0], a[1])
        elif op == "distinct":
            terms = [rec("BNOT", 1, rec("EQ", 1, a[i], a[j]))
                     for i in range(len(a)) for j in range(i + 1, len(a))]
            r = terms[0]
            for t in terms[1:]:
                r = rec("BAND", 1, r, t)
        elif op == "ite":
            r = rec("ITE", w, a[0], a[1], a[2])
        elif op == "concat":
            r, acc_w = a[0], n.args[0].width
            for x, arg in zip(a[1:], n.args[1:]):
                acc_w += arg.width
                r = rec("CONCAT", acc_w, r, x, p0=arg.width)
        elif op == "extract":
            hi, lo = n.params
            r = rec("EXTRACT", w, a[0], p1=lo)
        elif op == "zero_extend":
            r = rec("ZEXT", w, a[0])
        elif op == "sign_extend":
            r = rec("SEXT", w, a[0], p0=n.params[0])
        elif op == "array":
            r = rec("ARRVAR", w, p0=table(n.params[0], n.dom, w))
        elif op == "K":
            r = rec("KARR", w, a[0])
        elif op == "store":
            r = rec("STORE", w, a[0], a[1], a[2])
        elif op == "select":
            r = rec("SELECT", w, a[0], a[1])
        elif op == "apply":
            fname, dom = n.params
            r = rec("APPLY", w, a[0], p0=table(fname, dom, w))
        else:
            raise NotImplementedError(op)
        ix[n.id] = r
    S.roots = [ix[c.id] for c in constraints]
    return S


_libs = {}


def lib(wide: bool = False):
    """The C oracle: 512-bit values, or ``wide`` 1024-bit (a DAG with a node
    or table wider than 512 bits; the 512-bit build refuses one, rc -2)."""
    if wide not in _libs:
        path = _build.LIB_WIDE if wide else _build.LIB
        if not os.path.exists(path):
            _build.build()
        L = C.CDLL(path)
        p = C.c_void_p
        L.ev_run_gen.argtypes = [p, C.c_uint32, p, p, C.c_uint32, p, p, C.c_uint32, p, C.c_uint32,
                                 p, C.c_uint32, p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                 p, C.c_int]
        L.ev_run_leaves.argtypes = [p, C.c_uint32, p, p, C.c_uint32, p, p, C.c_uint32, C.c_uint32,
                                    p, C.c_uint64, p, p]
        L.ev_run_leaves_roots.argtypes = [p, C.c_uint32, p, p, C.c_uint32, p, p, C.c_uint32,
                                          C.c_uint32, p, C.c_uint64, p, C.c_int]
        L.ev_limbs.restype = C.c_int
        _libs[wide] = L
    return _libs[wide]


def _wide(S: Serialized) -> bool:
    w = max([r[1] for r in S.recs] + [t.key_w for t in S.tables] + [t.val_w for t in S.tables] +
            [0])
    return w > 512 or any(v >> 512 for v in S.consts)


def _arrays(S: Serialized):
    """(library, limbs, nodes, consts, tables, leafidx, roots)."""
    L = lib(_wide(S))
    nl = L.ev_limbs()
    nodes = np.ascontiguousarray(np.array(S.recs, dtype=np.uint32).reshape(-1, 8))
    consts = np.zeros((max(1, len(S.consts)), nl), dtype=np.uint64)
    for i, v in enumerate(S.consts):
        for k in range(nl):
            consts[i, k] = (v >> (64 * k)) & 0xFFFFFFFFFFFFFFFF
    tabs = (TableDesc * max(1, len(S.tables)))(*S.tables)
    leafidx = np.array(S.leafidx or [0], dtype=np.uint32)
    roots = np.array(S.roots or [0], dtype=np.uint32)
    return L, nl, nodes, consts, tabs, leafidx, roots


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def run_gen(S: Serialized, program, seed: int, prog_seed: int, first: int, n: int,
            threads: int = 0, pct=(50, 70, 85)) -> np.ndarray:
    L, nl, nodes, consts, tabs, leafidx, roots = _arrays(S)
    widths = np.array([l.width for l in program.leaves] or [1], dtype=np.uint32)
    pool = np.zeros((max(1, len(program.const_values)), nl), dtype=np.uint64)
    for i, v in enumerate(program.const_values):
        for k in range(4):
            pool[i, k] = (v >> (64 * k)) & 0xFFFFFFFFFFFFFFFF
    pctv = np.array(pct, dtype=np.uint32)
    out = np.zeros(n, dtype=np.uint8)
    rc = L.ev_run_gen(_p(nodes), nodes.shape[0], _p(consts), C.cast(tabs, C.c_void_p),
                          len(S.tables), _p(leafidx), _p(roots), len(S.roots), _p(widths),
                          len(program.leaves), _p(pool), len(program.const_values), _p(pctv),
                          seed & (2**64 - 1), prog_seed & (2**64 - 1), first, n, _p(out), threads)
    assert rc == 0, rc
    return out.astype(bool)


def run_leaves(S: Serialized, program, leaf_vals: Sequence[Sequence[int]], want_nodes=False):
    """leaf_vals: per assignment, the program's leaf values (<= 256 bits)."""
    L, nl_, nodes, consts, tabs, leafidx, roots = _arrays(S)
    n = len(leaf_vals)
    nl = len(program.leaves)
    lv = np.zeros((max(1, n), max(1, nl), 4), dtype=np.uint64)
    for a, vals in enumerate(leaf_vals):
        for i, v in enumerate(vals):
            for k in range(4):
                lv[a, i, k] = (v >> (64 * k)) & 0xFFFFFFFFFFFFFFFF
    vals_out = np.zeros((n, nodes.shape[0], nl_), dtype=np.uint64) if want_nodes else None
    out = np.zeros(max(1, n), dtype=np.uint8)
    rc = L.ev_run_leaves(_p(nodes), nodes.shape[0], _p(consts), C.cast(tabs, C.c_void_p),
                             len(S.tables), _p(leafidx), _p(roots), len(S.roots), nl, _p(lv), n,
                             None if vals_out is None else _p(vals_out), _p(out))
    assert rc == 0
    return out[:n].astype(bool), vals_out


def run_leaves_soa(S: Serialized, program, leaves_soa: np.ndarray, per_root: bool = False,
                   threads: int = 0) -> np.ndarray:
    """Root bits (``per_root``: (n, n_constraints) bits of every constraint)
    under the engine's own leaf buffer ((n_leaves, 8, n) u32 limbs, e.g.
    ``Engine.eval_gen(..., want_leaves=True)``)."""
    L, _, nodes, consts, tabs, leafidx, roots = _arrays(S)
    nl, _, n = leaves_soa.shape
    x = np.ascontiguousarray(leaves_soa.transpose(2, 0, 1)).astype(np.uint64)   # (n, nl, 8)
    lv = np.ascontiguousarray(x[:, :, 0::2] | (x[:, :, 1::2] << np.uint64(32)))  # (n, nl, 4)
    if nl == 0:
        lv = np.zeros((max(1, n), 1, 4), dtype=np.uint64)
    nr = max(1, len(S.roots))
    out = np.zeros((max(1, n), nr), dtype=np.uint8)
    rc = L.ev_run_leaves_roots(_p(nodes), nodes.shape[0], _p(consts),
                                   C.cast(tabs, C.c_void_p), len(S.tables), _p(leafidx), _p(roots),
                                   len(S.roots), max(nl, 1), _p(lv), n, _p(out), threads)
    assert rc == 0
    bits = out[:n, :len(S.roots)].astype(bool)
    return bits if per_root else bits.all(axis=1)


def node_value(vals_out, a: int, rec_index: int) -> int:
    v = 0
    for k in reversed(range(vals_out.shape[2])):
        v = (v << 64) | int(vals_out[a, rec_index, k])
    return v
