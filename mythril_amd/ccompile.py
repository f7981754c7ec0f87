"""Python side of the native host compiler (``include/mythcc.h``,
``mythril_amd/csrc/mg_compile.cpp``).

:func:`compile_native` takes the same arguments as
``ir.compile_constraints`` and returns the same :class:`ir.Program`: the
source DAG (hash-consed ``smt.node`` terms) is flattened into arrays in one
topological walk, the C++ compiler runs lowering, model construction
(search mode), scheduling, register allocation and the leaf pools, and the
result comes back as the instruction words, the constant table and a JSON
record of the rest.  ``tests/test_native_compiler.py`` checks that both
compilers emit identical programs.

The library is host code (g++, no GPU); it is built in-tree next to
``libmythgpu.so`` by ``mythril_amd/build.py`` and rebuilt on import when its
sources are newer."""

from __future__ import annotations

import collections.abc as _abc
import ctypes
import json
import os
import threading
from array import array
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import irdefs as I
from .smt.node import ARRAY, BOOL, topo_order

_lib = None
_lock = threading.Lock()
_OPS: Dict[str, int] = {}
_OTHER = 0

MGC_OK, MGC_UNSUPPORTED = 0, 1
_SORT = {"bv": 0, BOOL: 1, ARRAY: 2}
_REMAT = {"spill": 0, "always": 2}


class _Input(ctypes.Structure):
    _fields_ = [("n_nodes", ctypes.c_int32)] + \
        [(n, ctypes.c_void_p) for n in ("op", "sort", "width", "dom", "id", "arg_off", "args", "p0",
                                         "p1", "str", "cval_off", "cval")] + \
        [("strings", ctypes.c_char_p), ("n_strings", ctypes.c_int32),
         ("n_cons", ctypes.c_int32), ("cons", ctypes.c_void_p),
         ("n_probes", ctypes.c_int32), ("probes", ctypes.c_void_p),
         ("n_tables", ctypes.c_int32), ("table_name", ctypes.c_void_p),
         ("table_size", ctypes.c_void_p),
         ("default_entries", ctypes.c_int32), ("nreg", ctypes.c_int32),
         ("n_extra", ctypes.c_int32), ("extra", ctypes.c_void_p),
         ("leaf_pools", ctypes.c_int32), ("const_keys", ctypes.c_int32), ("solve", ctypes.c_int32),
         ("remat_mode", ctypes.c_int32), ("remat_k", ctypes.c_int32),
         ("keep_clean", ctypes.c_int32), ("search_hints", ctypes.c_int32),
         ("abi_presets", ctypes.c_int32), ("n_cval", ctypes.c_int32),
         ("n_string_bytes", ctypes.c_int32)]


def load():
    """The compiler library (built in-tree on first use)."""
    global _lib, _OTHER
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        from .build import build_compiler
        path = build_compiler()
        lib = ctypes.CDLL(path)
        lib.mgc_source_ops.restype = ctypes.c_char_p
        lib.mgc_compile.argtypes = [ctypes.POINTER(_Input), ctypes.POINTER(ctypes.c_void_p)]
        lib.mgc_compile.restype = ctypes.c_int
        lib.mgc_error.argtypes = [ctypes.c_void_p]
        lib.mgc_error.restype = ctypes.c_char_p
        lib.mgc_code.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)]
        lib.mgc_code.restype = ctypes.c_void_p
        lib.mgc_table.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32),
                                  ctypes.POINTER(ctypes.c_int32)]
        lib.mgc_table.restype = ctypes.c_void_p
        lib.mgc_meta.argtypes = [ctypes.c_void_p]
        lib.mgc_meta.restype = ctypes.c_char_p
        lib.mgc_free.argtypes = [ctypes.c_void_p]
        names = lib.mgc_source_ops().decode().split("\n")
        _OPS.update({n: i for i, n in enumerate(names)})
        _OTHER = _OPS["?"]
        _lib = lib
    return _lib


def _ptr(a):
    return ctypes.addressof(ctypes.c_char.from_buffer(a)) if len(a) else None


_ext = None


def _load_ext():
    """The CPython front-end (_mythcc: the compiler plus a C walk over the
    Node objects), built with the C-ABI library."""
    global _ext
    if _ext is None:
        import importlib.util
        from .build import cc_ext_path
        load()
        spec = importlib.util.spec_from_file_location("_mythcc", cc_ext_path())
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        _ext = mod
    return _ext


def compile_native(constraints: Sequence, probes: Sequence = (),
                   table_sizes: Optional[Dict[str, int]] = None, default_entries: int = 2,
                   nreg: int = I.NREG, extra_consts: Sequence[int] = (), leaf_pools: bool = False,
                   const_keys: bool = False, solve: bool = False, leaf_remat: Optional[str] = None,
                   keep_clean: Optional[bool] = None, search_hints: bool = False,
                   abi_presets: bool = False):
    """``ir.compile_constraints`` through the native compiler: the DAG is
    walked by the _mythcc front-end in C, compiled by mgc_compile."""
    from . import ir
    ext = _load_ext()
    M = (1 << 256) - 1
    extra = b"".join((v & M).to_bytes(32, "little") for v in extra_consts)
    remat = leaf_remat or ir.LEAF_REMAT
    mode = _REMAT.get(remat, 1)
    k = int(remat[7:]) if mode == 1 and remat[7:].isdigit() else 0
    rc, err, code_b, raw, ncv, meta = ext.compile(
        list(constraints), list(probes), _OPS, list((table_sizes or {}).items()), default_entries,
        nreg, extra, int(leaf_pools), int(const_keys), int(solve), mode, k,
        int(ir.KEEP_CLEAN if keep_clean is None else keep_clean), int(search_hints),
        int(abi_presets))
    if rc != MGC_OK:
        if rc == MGC_UNSUPPORTED:
            raise ir.Unsupported(err)
        raise RuntimeError("native compiler: " + err)
    prog = _program(np.frombuffer(code_b, dtype=np.uint32).reshape(-1, 4).copy(), raw, ncv,
                    json.loads(meta))
    prog.nreg = nreg
    return prog


def buckets(constraints: Sequence):
    """(independent-group label of each constraint, labels in order of first
    occurrence; DAG nodes per group): model.dependence_buckets' partition
    computed natively, with the size the compile-cost gate estimates from."""
    return _load_ext().buckets(list(constraints))


def flatten(constraints: Sequence, probes: Sequence = (),
            table_sizes: Optional[Dict[str, int]] = None, extra_consts: Sequence[int] = ()):
    """The mgc_input arrays of a DAG, built in Python (what another FFI host
    does): node arrays in topological order, the numerals' limbs, the
    NUL-separated names, constraint / probe / table indices, extra
    constants as 32-byte rows."""
    load()
    constraints, probes = list(constraints), list(probes)
    nodes = topo_order(constraints + probes)
    index = {n.id: i for i, n in enumerate(nodes)}
    ops, OTHER = _OPS, _OTHER
    f = {k: array("i") for k in ("op", "sort", "width", "dom", "str", "cval_off", "args")}
    f.update({k: array("q") for k in ("id", "p0", "p1")})
    f["arg_off"] = array("i", [0])
    cval = bytearray()
    strings: List[str] = []
    sidx: Dict[str, int] = {}

    def intern(s: str) -> int:
        k = sidx.get(s)
        if k is None:
            k = sidx[s] = len(strings)
            strings.append(s)
        return k
    for n in nodes:
        op = n.op
        code = ops.get(op, OTHER)
        f["op"].append(code)
        f["sort"].append(_SORT[n.sort])
        f["width"].append(n.width)
        f["dom"].append(n.dom or 0)
        f["id"].append(n.id)
        for a in n.args:
            f["args"].append(index[a.id])
        f["arg_off"].append(len(f["args"]))
        p0 = p1 = 0
        s = -1
        c = -1
        pr = n.params
        if op == "bvnum":
            c = len(cval) // 4
            cval += pr[0].to_bytes(4 * ((n.width + 31) // 32), "little")
        elif op in ("var", "array"):
            s = intern(pr[0])
        elif op == "apply":
            s = intern(pr[0])
            p0 = pr[1]
        elif op == "extract":
            p0, p1 = pr
        elif op in ("zero_extend", "sign_extend"):
            p0 = pr[0]
        elif code == OTHER:
            s = intern(op)
        f["p0"].append(p0)
        f["p1"].append(p1)
        f["str"].append(s)
        f["cval_off"].append(c)
    f["cons"] = array("i", [index[c.id] for c in constraints])
    f["probes"] = array("i", [index[p.id] for p in probes])
    tsz = table_sizes or {}
    f["table_name"] = array("i", [intern(k) for k in tsz])
    f["table_size"] = array("i", list(tsz.values()))
    M = (1 << 256) - 1
    f["extra"] = bytearray(b"".join((v & M).to_bytes(32, "little") for v in extra_consts))
    f["cval"] = bytearray(cval)
    f["strings"] = b"".join(s.encode() + b"\0" for s in strings)
    f["n_nodes"], f["n_strings"] = len(nodes), len(strings)
    return f


def compile_native_ctypes(constraints: Sequence, probes: Sequence = (),
                          table_sizes: Optional[Dict[str, int]] = None, default_entries: int = 2,
                          nreg: int = I.NREG, extra_consts: Sequence[int] = (),
                          leaf_pools: bool = False, const_keys: bool = False, solve: bool = False,
                          leaf_remat: Optional[str] = None, keep_clean: Optional[bool] = None,
                          search_hints: bool = False, abi_presets: bool = False):
    """The same compile through the plain C ABI (libmythcc.so, ctypes): the
    DAG flattened in Python (:func:`flatten`) into mgc_input arrays — what
    another FFI host does."""
    from . import ir
    lib = load()
    f = flatten(constraints, probes, table_sizes, extra_consts)
    remat = leaf_remat or ir.LEAF_REMAT
    mode = _REMAT.get(remat, 1)
    k = int(remat[7:]) if mode == 1 and remat[7:].isdigit() else 0
    P = {n: _ptr(f[n]) for n in ("op", "sort", "width", "dom", "id", "arg_off", "args", "p0", "p1",
                                  "str", "cval_off", "cval", "cons", "probes", "table_name",
                                  "table_size", "extra")}
    inp = _Input(f["n_nodes"], P["op"], P["sort"], P["width"], P["dom"], P["id"], P["arg_off"],
                 P["args"], P["p0"], P["p1"], P["str"], P["cval_off"], P["cval"], f["strings"],
                 f["n_strings"], len(f["cons"]), P["cons"], len(f["probes"]), P["probes"],
                 len(f["table_name"]), P["table_name"], P["table_size"], default_entries, nreg,
                 len(f["extra"]) // 32, P["extra"], int(leaf_pools), int(const_keys), int(solve),
                 mode, k, int(ir.KEEP_CLEAN if keep_clean is None else keep_clean),
                 int(search_hints), int(abi_presets), len(f["cval"]) // 4, len(f["strings"]))
    res = ctypes.c_void_p()
    rc = lib.mgc_compile(ctypes.byref(inp), ctypes.byref(res))
    try:
        if rc != MGC_OK:
            msg = lib.mgc_error(res).decode()
            if rc == MGC_UNSUPPORTED:
                raise ir.Unsupported(msg)
            raise RuntimeError("native compiler: " + msg)
        n = ctypes.c_int32()
        p = lib.mgc_code(res, ctypes.byref(n))
        code = np.frombuffer(ctypes.string_at(p, 16 * n.value), dtype=np.uint32).reshape(-1, 4).copy()
        rows, ncv = ctypes.c_int32(), ctypes.c_int32()
        p = lib.mgc_table(res, ctypes.byref(rows), ctypes.byref(ncv))
        raw = ctypes.string_at(p, 32 * rows.value) if rows.value else b""
        meta = json.loads(lib.mgc_meta(res))
    finally:
        lib.mgc_free(res)
    prog = _program(code, raw, ncv.value, meta)
    prog.nreg = nreg
    return prog


class LeafRecords(_abc.Sequence):
    """``Program.leaves`` of a native compile, decoded on first use: the
    compiler sends them as one string ("name TAB width TAB kind TAB source TAB
    chunk TAB entry" per line) plus their widths.  A search that misses —
    most compiles of a LASER stream — only needs the count and the widths
    (``model.search_leafgen``); a big search group has hundreds of leaves."""

    __slots__ = ("_rs", "_items", "widths")

    def __init__(self, rs: str, widths: Sequence[int]):
        self._rs = rs
        self._items = None
        self.widths = list(widths)

    def _decode(self):
        from .ir import Leaf
        items = []
        if self.widths:
            for line in self._rs.split("\n"):
                name, w, kind, source, chunk, entry = line.split("\t")
                items.append(Leaf(name, int(w), kind, source, int(chunk), int(entry)))
        self._items = items
        self._rs = None
        return items

    def __len__(self):
        return len(self.widths)

    def __getitem__(self, i):
        return (self._items if self._items is not None else self._decode())[i]

    def __iter__(self):
        return iter(self._items if self._items is not None else self._decode())

    def __eq__(self, other):
        return list(self) == list(other)

    def __repr__(self):
        return repr(list(self))

    def __reduce__(self):               # pickled (compile workers) as the list
        return (list, (list(self),))


def _program(code, raw: bytes, ncv: int, meta):
    from . import ir
    consts = np.frombuffer(raw, dtype="<u4").reshape(-1, 8).astype(np.uint32)
    const_values = [int.from_bytes(raw[32 * i:32 * i + 32], "little") for i in range(ncv)]
    Leaf = ir.Leaf
    if meta.get("leaves_rs") is not None:
        leaves = LeafRecords(meta["leaves_rs"], meta["leaf_widths"])
    else:
        leaves = [Leaf(*row) for row in meta["leaves"]]
    hist_counts = dict(meta["hist"])
    stats = {"lnodes": meta["lnodes"], "n_ins": int(code.shape[0]), "spills": meta["spills"],
             "reloads": meta["reloads"],
             "hist": {I.OPNAME[op]: hist_counts[op] for op in meta["hist_order"]}}
    prog = ir.Program(code, consts, const_values, leaves, meta["n_lds"], meta["n_probes"],
                      meta["n_roots"], dict(meta["table_sizes"]), dict(meta["table_kinds"]),
                      {k: [int(h, 16) for h in v] for k, v in meta["table_ckeys"]}, stats,
                      [tuple(r) for r in meta["pool_ranges"]], dict(meta["derived"]),
                      {k: v for k, v in meta["entry_keys"]}, meta["n_user_probes"])
    # native compile phases (us): decode, lower, solve, sinks, schedule,
    # allocate, pools, metadata — diagnostics only (tools/compile_profile.py)
    prog.compile_us = meta.get("t_us")
    pre = meta.get("presets")
    if pre is not None:
        from .abi import Plan
        prog.presets = Plan(vars={k: int(v, 16) for k, v in pre["vars"]},
                            arrays={k: dict(cells) for k, cells in pre["arrays"]})
    return prog
