"""Drop-in replacement of ``mythril.support.model.get_model``
(reference ``mythril/support/model.py:15-49``).

Contract kept from the reference, in the same order:

1. ``@lru_cache(maxsize=2**23)`` keyed on (constraints, minimize, maximize,
   enforce_execution_time);
2. timeout = ``args.solver_timeout`` (ms), clipped to the execution time left
   minus 500 ms when ``enforce_execution_time``; ``<= 0`` → ``UnsatError``
   before any work (``model.py:26-31``);
3. a Python ``False`` constraint → ``UnsatError``; Python bools are dropped
   (``model.py:32-36``);
4. z3 ``unknown`` is treated as UNSAT (``model.py:47-49``).

Routing:

* ``minimize``/``maximize`` non-empty (only ``analysis/solver.py:65``) →
  stock z3 ``Optimize``: the reported transaction sequence depends on the
  optimum, so the GPU never answers these.
* otherwise → compile the DAG (``mythril_amd.ir``), GPU witness search
  (``mg_search``); a witness is re-verified by z3 when z3 is present and a
  genuine z3 model is returned; on a miss, an unsupported operator or any
  engine error → stock z3.  **UNSAT is only ever concluded by z3**: without
  z3 a miss raises :class:`SolverUnavailable`, never ``UnsatError``.
"""

from __future__ import annotations

import logging
import time

import numpy as np
from functools import lru_cache
from typing import Dict, List, Optional, Sequence

from . import z3bridge
from .assign import Assignment, unpack
from .engine import EngineError, EngineUnavailable, LeafGen, device_slots, get_engine
from . import irdefs as I
from .ir import Program, Unsupported, compile_constraints, harvest_hints  # noqa: F401
from .smt import node as N

log = logging.getLogger(__name__)

try:  # inside a Mythril installation use its exception and singletons
    from mythril.exceptions import UnsatError  # type: ignore
except Exception:  # noqa: BLE001 - z3/mythril absent here
    class UnsatError(Exception):
        """Mirror of ``mythril.exceptions.UnsatError`` (``exceptions.py:16-20``)."""


class SolverUnavailable(RuntimeError):
    """No witness found on the GPU and no z3 to conclude UNSAT."""


class Args:
    """Mirror of ``mythril.support.support_args.Args`` (``support_args.py:1-16``)."""

    def __init__(self):
        self.solver_timeout = 10000
        self.sparse_pruning = True
        self.unconstrained_storage = False
        self.parallel_solving = False
        self.call_depth_limit = 3
        self.iprof = True


class TimeHandler:
    """Mirror of ``laser/ethereum/time_handler.py:5-18``."""

    def __init__(self):
        self._start_time = int(time.time() * 1000)
        self._execution_time = 86400 * 1000

    def start_execution(self, execution_time):
        self._start_time = int(time.time() * 1000)
        self._execution_time = execution_time * 1000

    def time_remaining(self):
        return self._execution_time - (int(time.time() * 1000) - self._start_time)


args = Args()
time_handler = TimeHandler()


PHASES = ("flatten", "refute", "compile", "load", "search", "verify")


class SolverStatistics:
    """``SolverStatistics`` (``solver_statistics.py:29-43``: query count and z3
    time, counted while ``enabled``) plus the pre-filter's own counters and a
    per-phase time breakdown of the GPU path (seconds).  ``install()`` makes
    Mythril's own singleton print these lines too, where ``fire_lasers`` logs
    it (``mythril_analyzer.py:181``)."""

    def __init__(self):
        self.enabled = False
        self.query_count = 0
        self.solver_time = 0.0
        self.reset_gpu()

    def reset_gpu(self):
        self.gpu_queries = 0
        self.gpu_hits = 0
        self.gpu_candidates = 0
        self.gpu_time = 0.0
        self.kernel_time = 0.0          # device time of the search launches (HIP events)
        self.witness_time = 0.0         # part of the search phase: witnesses read back and unpacked
        self.memo_misses = 0            # queries answered "miss" by the group-miss memo
        self.gated = 0                  # queries whose compile estimate exceeded the budget
        self.shape_skipped = 0          # queries of a shape the search keeps missing
        self.fallbacks = 0
        self.unsupported = 0
        self.errors = 0
        self.rejected = 0
        self.ground_true = 0            # groups folded to true: answered without a launch
        self.ground_false = 0           # queries with a group folded to false: not searched
        self.refuted = 0                # queries refuted on the host (refute.py): not compiled
        self.phase = {k: 0.0 for k in PHASES}

    def gpu_report(self) -> str:
        return ("GPU pre-filter: queries: {} hits: {} fallbacks: {} unsupported: {} errors: {} "
                "rejected by z3: {} memo misses: {} compile-gated: {} shape-skipped: {} "
                "refuted: {}\n"
                "GPU candidates: {} time: {:.3f}s (kernel {:.3f}s; {})").format(
            self.gpu_queries, self.gpu_hits, self.fallbacks, self.unsupported, self.errors,
            self.rejected, self.memo_misses, self.gated, self.shape_skipped, self.refuted,
            self.gpu_candidates,
            self.gpu_time,
            self.kernel_time, ", ".join("%s %.3fs" % (k, self.phase[k]) for k in PHASES))

    def __repr__(self):
        return "Query count: {} \nSolver time: {}\n{}".format(self.query_count, self.solver_time,
                                                              self.gpu_report())


class _Phase:
    """``with _Phase("compile"):`` adds the block's wall time to the phase."""

    def __init__(self, name: str):
        self.name = name

    def __enter__(self):
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        stats.phase[self.name] += time.perf_counter() - self.t0
        return False


def _count_kernel(eng) -> None:
    """Device time of the engine's last search (HIP events around its
    launches inside libmythgpu, ``mg_last_kernel_ms``)."""
    ms = getattr(eng, "last_kernel_ms", None)
    if ms is not None:
        stats.kernel_time += ms() / 1000.0


stats = SolverStatistics()

# candidate budget per query (device-generated, counter-based streams) and
# the wall-time share of the query's timeout the GPU search may use.  The
# cap bounds what a MISS costs before z3 decides the query: round 4's census
# of 1292 witnesses over 1389 distinct stand-in queries found every first
# index below 2^16 (max 59505; profiles/r04/hit_index_census_r4h.log), so
# 2^20 keeps 16x headroom at a quarter of the old 2^22 miss cost
SEARCH_CANDIDATES = 1 << 20
SEARCH_SEED = 0x6D797468
SEARCH_BUDGET_MS = 200
# conservative engine throughput (IR instructions x candidates per second)
# used to size a search so it fits its time budget (one device launch
# sequence cannot be interrupted)
INS_CAND_PER_S = 3.0e11
# devices the batched search spreads programs over (corpus axis)
DEVICES = [0]
GPU_ENABLED = True
# adaptive gate (see _shape_gate): after SHAPE_MIN searches of one query
# shape with a hit rate below SHAPE_FLOOR, only every SHAPE_PROBE-th query of
# that shape is searched
SHAPE_GATE = True
REFUTE = True              # host refutation before compiling (refute.py)
SHAPE_MIN, SHAPE_FLOOR, SHAPE_PROBE = 4, 1.0 / 16, 8


def configure_from_env(env=None) -> None:
    """Pre-filter configuration from the environment:
    ``MYTHRIL_GPU=0`` turns the GPU path off (every query goes to z3),
    ``MYTHRIL_GPU_DEVICES=0,1,...`` the devices batched searches use,
    ``MYTHRIL_GPU_CANDIDATES`` the candidates per query (a power of two),
    ``MYTHRIL_GPU_BUDGET_MS`` the share of a query's timeout the search may
    take, ``MYTHRIL_GPU_ADAPTIVE=0`` turns the per-shape gate off,
    ``MYTHRIL_GPU_REFUTE=0`` the host refutation (refute.py)."""
    global GPU_ENABLED, DEVICES, SEARCH_CANDIDATES, SEARCH_BUDGET_MS, SHAPE_GATE, REFUTE
    import os
    env = os.environ if env is None else env
    GPU_ENABLED = env.get("MYTHRIL_GPU", "1").strip().lower() not in ("0", "off", "false", "no")
    devs = env.get("MYTHRIL_GPU_DEVICES", "").strip()
    if devs:
        DEVICES = [int(d) for d in devs.split(",") if d.strip()]
    if env.get("MYTHRIL_GPU_CANDIDATES"):
        n = max(1, int(env["MYTHRIL_GPU_CANDIDATES"]))
        SEARCH_CANDIDATES = 1 << (n.bit_length() - 1)
    if env.get("MYTHRIL_GPU_BUDGET_MS"):
        SEARCH_BUDGET_MS = max(0.0, float(env["MYTHRIL_GPU_BUDGET_MS"]))
    SHAPE_GATE = env.get("MYTHRIL_GPU_ADAPTIVE", "1").strip().lower() not in ("0", "off", "false",
                                                                             "no")
    REFUTE = env.get("MYTHRIL_GPU_REFUTE", "1").strip().lower() not in ("0", "off", "false", "no")


configure_from_env()


class Model:
    """Result of :func:`get_model`.  Wraps z3 models when z3 verified the
    witness (same interface as ``laser/smt/model.py``), otherwise the GPU
    witness itself (``assignment``)."""

    def __init__(self, models: Optional[List[object]] = None,
                 assignment: Optional[Assignment] = None, programs=None):
        self.raw = models or []
        self.assignment = assignment
        if isinstance(programs, Program):
            programs = [programs]
        self.programs = list(programs or [])
        self.table_sizes: Dict[str, int] = {}
        for p in self.programs:
            self.table_sizes.update(p.table_sizes)
        if assignment is not None:     # constant-keyed entries count too
            for name, (entries, _) in list(assignment.arrays.items()) + list(assignment.funcs.items()):
                self.table_sizes[name] = max(self.table_sizes.get(name, 0), len(entries))

    def decls(self):
        out = []
        for m in self.raw:
            out.extend(m.decls())
        return out

    def __getitem__(self, item):
        """``laser/smt/model.py:27-43``: the first internal model with an
        interpretation; an IndexError of the last model propagates.  A
        witness-only model (no z3) answers variable names from the witness."""
        for i, m in enumerate(self.raw):
            try:
                r = m[item]
                if r is not None:
                    return r
            except IndexError:
                if i == len(self.raw) - 1:
                    raise
                continue
        if not self.raw and self.assignment is not None and isinstance(item, str):
            return self.assignment.vars.get(item)
        return None

    def eval(self, expression, model_completion: bool = False):
        if self.raw:
            for i, m in enumerate(self.raw):
                if expression.decl() in list(m.decls()) or i == len(self.raw) - 1:
                    return m.eval(expression, model_completion)
            return None
        return self.eval_node(expression if isinstance(expression, N.Node) else expression.raw)

    def eval_node(self, node: N.Node) -> int:
        """Evaluate a DAG under the witness — on the GPU (one lane)."""
        if self.assignment is None:
            raise ValueError("no witness")
        from .assign import pack
        prog = compile_constraints([], [node], table_sizes=dict(self.table_sizes) or None)
        eng = get_engine()
        lp = eng.load(prog)
        _, probes = eng.eval(lp, pack(prog, [self.assignment]), want_probes=True)
        v = 0
        for k in reversed(range(prog.n_probes)):
            for j in reversed(range(8)):
                v = (v << 32) | int(probes[k, j, 0])
        return v


def _raw_nodes(constraints) -> List[N.Node]:
    """laser.smt Bool objects → DAG nodes (z3 ASTs are flattened)."""
    out = []
    memo: Dict[int, N.Node] = {}
    for c in constraints:
        raw = getattr(c, "raw", c)
        if isinstance(raw, N.Node):
            out.append(raw)
        else:
            out.append(z3bridge.to_node(raw, memo))
    return out


def search_leafgen(prog: Program) -> List[LeafGen]:
    """Candidate generator for witness search: 20 % uniform, 20 % small,
    20 % boundary values, 40 % pool values (+-1).  A program compiled with
    leaf_pools draws each leaf's pool values from the constants it is
    compared with (ir._leaf_pools); otherwise from every constant of the
    query."""
    n_c = len(prog.const_values)
    # (the widths alone: a native compile's leaves are decoded only when a
    # witness is unpacked, ccompile.LeafRecords)
    widths = getattr(prog.leaves, "widths", None) or [l.width for l in prog.leaves]
    if prog.pool_ranges:
        return [LeafGen(w, off, n, 20, 40, 60) for w, (off, n) in zip(widths, prog.pool_ranges)]
    return [LeafGen(w, 0, n_c, 20, 40, 60) for w in widths]


_SEARCH_CACHE: "OrderedDict[tuple, Program]" = None
SEARCH_CACHE_SIZE = 2048


def _compile_search(nodes: Sequence[N.Node], probes: Sequence[N.Node] = ()) -> Program:
    """Search program of an independent group, cached: LASER's path
    constraints grow one JUMPI at a time, so sibling and successive
    ``is_possible`` queries share most of their groups (hash-consed nodes:
    a group is identified by its node ids).  Compiled by
    :func:`_compile_search_uncached`."""
    global _SEARCH_CACHE
    from collections import OrderedDict
    if _SEARCH_CACHE is None:
        _SEARCH_CACHE = OrderedDict()
    key = (tuple(n.id for n in nodes), tuple(p.id for p in probes))
    prog = _SEARCH_CACHE.get(key)
    if prog is not None:
        _SEARCH_CACHE.move_to_end(key)
        return prog
    prog = _compile_search_uncached(nodes, probes)
    prog.group_key = _group_key(nodes)
    _SEARCH_CACHE[key] = prog
    if len(_SEARCH_CACHE) > SEARCH_CACHE_SIZE:
        _SEARCH_CACHE.popitem(last=False)
    return prog


def _compile_search_uncached(nodes: Sequence[N.Node], probes: Sequence[N.Node] = ()) -> Program:
    """Search program: solve mode (part of the model constructed), or — when
    its argument-keyed entries keep too many values live for the spill
    budget — the plain search form (every model value generated).
    ``probes`` are evaluated under each candidate's model."""
    try:
        # candidate hints from the query's numerals, ABI offsets pinned
        # (abi.py: a witness carries the presets, Program.presets)
        return compile_constraints(nodes, probes, leaf_pools=True, const_keys=True, solve=True,
                                   search_hints=True, abi_presets=True)
    except Unsupported as e:
        if "spill budget" not in str(e):
            raise
        return compile_constraints(nodes, probes, leaf_pools=True, const_keys=True,
                                   search_hints=True)


def _witness(eng, lp, hit) -> Assignment:
    """The model of a search hit (index, leaves[, probes]): a solve-mode
    program also reports the values it computed — the probes the batched
    search regenerated with the leaves, or those of one re-evaluated lane."""
    idx, leaves = hit[0], hit[1]
    prog = getattr(lp, "program", lp)
    if prog.solved:
        if len(hit) > 2 and hit[2] is not None:
            return unpack(prog, leaves, hit[2])
        leaves, probes = eng.witness(lp, SEARCH_SEED, idx)
        return unpack(prog, leaves, probes)
    return unpack(prog, leaves)


_SYMS: "Dict[int, frozenset]" = {}
_SYMS_SIZE = 1 << 16


def _symbols(c: N.Node) -> frozenset:
    """Free symbols under one constraint, memoised by node id (nodes are
    immutable and ids never reused: LASER re-asks the same path constraints
    on every JUMPI, so a stream walks each constraint once)."""
    hit = _SYMS.get(c.id)
    if hit is None:
        hit = frozenset((n.op == "var", n.params[0]) for n in N.topo_order([c])
                        if n.op in ("var", "array", "apply"))
        if len(_SYMS) >= _SYMS_SIZE:
            _SYMS.clear()
        _SYMS[c.id] = hit
    return hit


def dependence_buckets(nodes: Sequence[N.Node]) -> List[List[N.Node]]:
    """Split constraints into groups that share no free symbol — the
    ``DependenceMap`` of ``IndependenceSolver``
    (``mythril/laser/smt/solver/independence_solver.py:38-84``), with free
    arrays and uninterpreted functions counted as symbols too (the reference
    only counts expression leaves; a GPU witness is a joint table per array /
    UF, so two groups reading one table are not independent here).  Groups
    keep the constraints' order; a symbol-free constraint is its own group.
    The native front-end computes the same partition in one walk
    (``_mythcc.buckets``); :func:`dependence_buckets_py` is its
    specification."""
    return dependence_buckets_sized(nodes)[0]


def dependence_buckets_sized(nodes: Sequence[N.Node]):
    """(:func:`dependence_buckets`, DAG nodes per group) — the size is what
    the compile-cost gate prices (``COMPILE_MS_PER_NODE``)."""
    from . import ir
    nodes = list(nodes)
    if ir.COMPILER != "py":
        from .ccompile import buckets
        labels, sizes = buckets(nodes)
        out: List[List[N.Node]] = []
        for c, g in zip(nodes, labels):
            if g == len(out):
                out.append([])
            out[g].append(c)
        return out, sizes
    out = dependence_buckets_py(nodes)
    return out, [len(N.topo_order(b)) for b in out]


def dependence_buckets_py(nodes: Sequence[N.Node]) -> List[List[N.Node]]:
    """:func:`dependence_buckets` in Python (the specification)."""
    parent: Dict[object, object] = {}

    def find(k):
        while parent[k] != k:
            parent[k] = parent[parent[k]]
            k = parent[k]
        return k

    for i, c in enumerate(nodes):
        syms = _symbols(c)
        parent.setdefault(("c", i), ("c", i))
        for sym in syms:
            parent.setdefault(sym, sym)
            a, b = find(("c", i)), find(sym)
            if a != b:
                parent[b] = a
    groups: Dict[object, List[N.Node]] = {}
    for i, c in enumerate(nodes):
        groups.setdefault(find(("c", i)), []).append(c)
    return list(groups.values())


def _merge(parts: Sequence[Assignment]) -> Assignment:
    out = Assignment()
    for a in parts:
        out.vars.update(a.vars)
        out.arrays.update(a.arrays)
        out.funcs.update(a.funcs)
    return out


def _n_cand(progs: Sequence[Program], budget_ms: float) -> int:
    """Candidates that fit the time budget (power of two, <= SEARCH_CANDIDATES)."""
    ins = max(1, sum(p.n_ins for p in progs))
    n = int(max(budget_ms, 0.0) / 1000.0 * INS_CAND_PER_S / ins)
    n = min(SEARCH_CANDIDATES, max(1 << 16, n))
    return 1 << (n.bit_length() - 1)


GROUND_MISS = 1 << 62     # group-miss depth of a group that folds to false


def _ground_value(p: Program) -> Optional[bool]:
    """False when a root of the group folded to the constant false (a CONST
    instruction carrying the ROOT flag: no candidate can satisfy it, whatever
    the other roots); True when the whole group folded to the constant true
    (its one instruction, no leaf and no ABI preset left: nothing for a
    candidate to choose); else None.  Such a group needs no launch: true
    joins every witness as is, false sends the query to z3."""
    w0 = p.code[:, 0]
    for k in np.flatnonzero(((w0 & 0xFF) == I.CONST) & ((w0 & I.ROOT_FLAG) != 0)):
        if not int(p.consts[int(p.code[k, 2]), 0]) & 1:
            return False
    if p.n_ins == 1 and not p.leaves and not p.presets and (int(w0[0]) & 0xFF) == I.CONST:
        return True
    return None


def search_groups(progs: Sequence[Program], n_cand: int):
    """``batch_search_devices`` over the groups that need a search: a group
    folded to a constant (:func:`_ground_value`) is answered on the host —
    true: (0, empty model); false: (-1, None) — and nothing is launched for
    any group of a query with a false one (round 4: 2 of 3 C3 stand-in groups
    fold to true; every one was a load + launch + witness read)."""
    return _search_sets([progs], n_cand)


# How _search_sets answered a group (its ``kinds`` list): launched, folded to
# a constant on the host, or skipped because a sibling group of its query
# folded to false.
SEARCHED, GROUND_TRUE, GROUND_FALSE, SKIPPED = "searched", "true", "false", "skipped"


def _search_sets(sets: Sequence[Sequence[Program]], n_cand: int,
                 kinds: Optional[List[str]] = None):
    """:func:`search_groups` over several queries' groups in ONE batched
    search: a query with a group folded to false contributes no launch.
    ``kinds`` (when given) receives, per group in output order, how it was
    answered — only SEARCHED and GROUND_FALSE misses say anything about the
    group itself (a SKIPPED group was never searched)."""
    ground = [[_ground_value(p) for p in progs] for progs in sets]
    dead = [any(g is False for g in gs) for gs in ground]
    stats.ground_false += sum(dead)
    live = [p for progs, gs, d in zip(sets, ground, dead) if not d
            for p, g in zip(progs, gs) if g is None]
    stats.ground_true += sum(g is True for gs, d in zip(ground, dead) if not d for g in gs)
    found = iter(batch_search_devices(live, n_cand) if live else ())
    out = []
    for gs, d in zip(ground, dead):
        for g in gs:
            if g is False:
                kind, r = GROUND_FALSE, (-1, None)
            elif d:
                kind, r = SKIPPED, (-1, None)
            elif g is None:
                kind, r = SEARCHED, next(found)
            else:
                kind, r = GROUND_TRUE, (0, Assignment())
            out.append(r)
            if kinds is not None:
                kinds.append(kind)
    return out


def batch_search_devices(progs: Sequence[Program], n_cand: int):
    """``Engine.batch_search`` over ``DEVICES``: programs are spread over the
    devices by longest-processing-time first on their instruction counts
    (the corpus axis, mythril_amd/shard.py), each device searches its share
    in its own host thread (the C ABI releases the GIL; one context per
    device), and the results come back in program order as
    (first index, witness Assignment) or (-1, None).  A single program on
    several devices is split on the assignment axis instead
    (:func:`search_assignment_axis`)."""
    from .shard import lpt_assign
    devices = list(DEVICES) or [0]
    if len(progs) == 1 and len(devices) > 1:
        return [search_assignment_axis(progs[0], n_cand, devices)]
    if len(devices) == 1 or len(progs) < 2:
        eng = get_engine(devices[0])
        with _Phase("load"):
            loaded = [eng.load(p, search_leafgen(p), prog_seed=0) for p in progs]
        with _Phase("search"):
            hits = eng.batch_search(loaded, SEARCH_SEED, n_cand, want_probes=True)
            _count_kernel(eng)
            t0 = time.perf_counter()
            out = [(h[0], _witness(eng, lp, h) if h[0] >= 0 else None)
                   for lp, h in zip(loaded, hits)]
            stats.witness_time += time.perf_counter() - t0
            return out
    parts = lpt_assign([float(p.n_ins) for p in progs], len(devices))
    out: List = [None] * len(progs)

    def run(dev, idx):
        eng = get_engine(*dev)
        loaded = [eng.load(progs[i], search_leafgen(progs[i]), prog_seed=0) for i in idx]
        hits = eng.batch_search(loaded, SEARCH_SEED, n_cand, want_probes=True)
        _count_kernel(eng)
        for i, lp, h in zip(idx, loaded, hits):
            out[i] = (h[0], _witness(eng, lp, h) if h[0] >= 0 else None)
    with _Phase("search"):
        _on_devices(run, [(d, idx) for d, idx in zip(device_slots(devices), parts) if idx])
    return out


def _on_devices(fn, jobs) -> None:
    """Run ``fn(*job)`` for every job, one host thread per job (one device
    context each; the C ABI releases the GIL); the first error re-raises."""
    import threading
    errors: List[BaseException] = []

    def body(*a):
        try:
            fn(*a)
        except BaseException as e:  # noqa: BLE001 - re-raised in the caller
            errors.append(e)
    threads = [threading.Thread(target=body, args=job) for job in jobs]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        raise errors[0]


def search_assignment_axis(prog: Program, n_cand: int, devices: Sequence[int]):
    """One program's candidate range split over devices (SURVEY §8e
    assignment axis): device g searches candidate indices
    [g*n/G, (g+1)*n/G) of the same counter-based stream, and the host
    reduces MIN over the devices' first satisfying indices — the index a
    single-device sweep of [0, n) returns (the ranges are ordered and
    disjoint).  Only the seed and the range travel; the winning witness is
    regenerated on the device that found it."""
    G = len(devices)
    bounds = [n_cand * g // G for g in range(G + 1)]
    res: List = [None] * G

    def run(g, dev):
        eng = get_engine(*dev)
        lp = eng.load(prog, search_leafgen(prog), prog_seed=0)
        n = bounds[g + 1] - bounds[g]
        h = eng.search(lp, SEARCH_SEED, n, first_index=bounds[g]) if n else (-1, None)
        _count_kernel(eng)
        res[g] = (h[0], _witness(eng, lp, h) if h[0] >= 0 else None)
    with _Phase("search"):
        _on_devices(run, list(enumerate(device_slots(devices))))
    found = [r for r in res if r[0] >= 0]
    return min(found, key=lambda r: r[0]) if found else (-1, None)


# Group-miss memo.  A group's search program, leaf generator and candidate
# streams are functions of its constraint nodes alone (hash-consed ids), so
# a group that missed on candidates [0, N) misses again on any [0, n <= N):
# such a query is answered "miss" without compiling or launching anything.
# A group that EXTENDS a missed group (LASER appends one JUMPI condition at a
# time, so successive is_possible groups grow) is not searched either: the
# superset is satisfiable only where the subset is, and the subset's search
# already failed — z3 decides it, as it decides every miss.  This never
# changes an answer (UNSAT is only concluded by z3), only where the time goes.
GROUP_MISS_SIZE = 1 << 14
SUPERSET_SKIP = True
_group_miss: "Dict[frozenset, int]" = {}
_miss_index: "Dict[int, List[frozenset]]" = {}
# compile-cost gate: estimated host compile time per DAG node of an uncached
# group — native compiler: 2.5 ms for the ~990-node C3 queries on the GPU
# box (profiles/r03/search_r3_native.log); the Python one (MYTHRIL_GPU_
# COMPILER=py) measured ~0.035 ms/node
COMPILE_MS_PER_NODE = 0.004
COMPILE_MS_PER_NODE_PY = 0.04


def _group_key(nodes: Sequence[N.Node]) -> frozenset:
    return frozenset(n.id for n in nodes)


def _known_miss(key: frozenset, n_cand: int) -> bool:
    if _group_miss.get(key, -1) >= n_cand:
        return True
    if not SUPERSET_SKIP:
        return False
    for c in key:
        for m in _miss_index.get(c, ()):
            # a proper subset missed, searched at least as far as this query
            # would be (a small batch_is_possible miss must not stop a full
            # get_model search of its supersets)
            if len(m) < len(key) and m <= key and _group_miss.get(m, -1) >= n_cand:
                return True
    return False


def _note_miss(key: frozenset, n_cand: int) -> None:
    if key in _group_miss:
        _group_miss[key] = max(_group_miss[key], n_cand)
        return
    if len(_group_miss) >= GROUP_MISS_SIZE:
        old = next(iter(_group_miss))
        del _group_miss[old]
        lst = _miss_index.get(min(old), [])
        if old in lst:
            lst.remove(old)
    _group_miss[key] = n_cand
    if key:
        _miss_index.setdefault(min(key), []).append(key)


# Adaptive gate.  LASER asks the same KIND of question again and again: a
# module's check at one instruction (an overflow test, an ``ISZERO`` of a
# selector comparison) is the newest constraint of every query it makes, on
# every path that reaches the instruction.  Behind SafeMath such checks are
# unsatisfiable on every path, so searching them only adds compile time to a
# z3 call that has to happen anyway.  The gate keeps hit / miss counts per
# shape of the newest constraint (its operator tree to depth 3, leaves by
# kind); once a shape has been searched SHAPE_MIN times with a hit rate below
# SHAPE_FLOOR, only every SHAPE_PROBE-th query of it is searched (so a shape
# that starts to hit is noticed again).  Like the memo it never changes an
# answer — a skipped query goes to z3, as stock Mythril's does — only where
# the time goes.
_shape_stats: "Dict[str, List[int]]" = {}     # shape -> [searches, hits, skipped since probe]
_SHAPE_DEPTH = 3


def query_shape(c: N.Node, depth: int = _SHAPE_DEPTH) -> str:
    """Operator tree of ``c`` to ``depth`` (numerals as ``k``, other leaves
    by kind and width): constraints a module builds at one instruction on
    different paths share it."""
    if depth == 0 or not c.args:
        if c.op == "bvnum":
            return "k%d" % c.width
        return "%s%d" % (c.op, c.width or 0)
    return "%s(%s)" % (c.op, ",".join(query_shape(a, depth - 1) for a in c.args))


def _shape_gate(shape: str) -> bool:
    """True when the query should be searched."""
    if not SHAPE_GATE:
        return True
    st = _shape_stats.get(shape)
    if st is None or st[0] < SHAPE_MIN or st[1] >= SHAPE_FLOOR * st[0]:
        return True
    st[2] += 1
    if st[2] >= SHAPE_PROBE:
        st[2] = 0
        return True
    return False


def _shape_note(shape: str, hit: bool) -> None:
    st = _shape_stats.setdefault(shape, [0, 0, 0])
    st[0] += 1
    st[1] += int(hit)
    if len(_shape_stats) > GROUP_MISS_SIZE:
        _shape_stats.pop(next(iter(_shape_stats)))


def clear_search_memos() -> None:
    """Forget compiled groups, group misses and shape statistics
    (tools/search_bench.py's cold runs)."""
    global _SEARCH_CACHE
    _SEARCH_CACHE = None
    _group_miss.clear()
    _miss_index.clear()
    _shape_stats.clear()


def _compile_estimate_ms(buckets, sizes) -> float:
    from . import ir
    cache = _SEARCH_CACHE or {}
    n = sum(sz for b, sz in zip(buckets, sizes) if (tuple(c.id for c in b), ()) not in cache)
    return n * (COMPILE_MS_PER_NODE_PY if ir.COMPILER == "py" else COMPILE_MS_PER_NODE)


def _refuted_group(buckets, keys) -> Optional[frozenset]:
    """Key of the first group the host refutes (refute.refuted), or None.
    One-constraint groups are skipped: the compiler folds a ground one, and
    a single atom has no partner to contradict."""
    if not REFUTE:
        return None
    from .refute import refuted
    for b, k in zip(buckets, keys):
        if len(b) > 1 and refuted(b):
            return k
    return None


def gpu_search(nodes: Sequence[N.Node], budget_ms: float):
    """(assignment, programs) of a satisfying candidate, or None.  Queries
    that split into independent groups (dependence_buckets) search every
    group in one batched launch sequence and join the group witnesses, so the
    hit probability is per group rather than their product.  The candidate
    count is sized to ``budget_ms``; the whole range runs on the device with
    no host round trip (mg_search / mg_batch_search).  The group-miss memo
    answers repeated (or extended) missed groups at once, and a query whose
    estimated compile time exceeds the budget is not searched."""
    buckets, sizes = dependence_buckets_sized(nodes)
    keys = [_group_key(b) for b in buckets]
    if any(_known_miss(k, SEARCH_CANDIDATES) for k in keys):
        stats.memo_misses += 1
        return None
    # a group whose atoms contradict each other (refute.py: SafeMath's
    # require against the module's check on the same terms) is not compiled
    # or searched; z3 still decides the query, so UNSAT stays z3's
    with _Phase("refute"):
        dead = _refuted_group(buckets, keys)
    if dead is not None:
        stats.refuted += 1
        _note_miss(dead, GROUND_MISS)
        return None
    shape = query_shape(nodes[-1]) if nodes else ""
    if not _shape_gate(shape):
        stats.shape_skipped += 1
        return None
    if _compile_estimate_ms(buckets, sizes) > budget_ms:
        stats.gated += 1
        return None
    with _Phase("compile"):
        progs = [_compile_search(b) for b in buckets]
    n_cand = _n_cand(progs, budget_ms)
    if any(_known_miss(k, n_cand) for k in keys):
        stats.memo_misses += 1
        return None
    devices = list(DEVICES) or [0]
    ground = [_ground_value(p) for p in progs]
    if any(g is False for g in ground):
        stats.ground_false += 1
        for k, g in zip(keys, ground):
            if g is False:
                _note_miss(k, GROUND_MISS)
        return None
    if len(progs) > 1 or len(devices) > 1 or ground[0] is not None:
        hits = search_groups(progs, n_cand)
    else:
        eng = get_engine(devices[0])
        with _Phase("load"):
            lp = eng.load(progs[0], search_leafgen(progs[0]), prog_seed=0)
        with _Phase("search"):
            h = eng.search(lp, SEARCH_SEED, n_cand)
            _count_kernel(eng)
            hits = [(h[0], _witness(eng, lp, h) if h[0] >= 0 else None)]
    stats.gpu_candidates += sum(n_cand if i < 0 else i + 1 for i, _ in hits)
    for k, (i, _) in zip(keys, hits):
        if i < 0:
            _note_miss(k, n_cand)
    _shape_note(shape, all(i >= 0 for i, _ in hits))
    if any(i < 0 for i, _ in hits):
        return None
    return _merge([a for _, a in hits]), progs


# Set by install(): the reference's own Optimize wrapper
# (mythril/laser/smt/solver/solver.py:86-105, timed by @stat_smt_query) and
# Model class (laser/smt/model.py), so inside Mythril the fallback is
# literally the stock code path and a GPU answer is a stock Model.
_stock_optimize = None
_stock_model = None


def _z3_check(constraints, minimize, maximize, timeout):
    """Stock path: z3 Optimize, exactly as the reference."""
    if _stock_optimize is not None:
        s = _stock_optimize()
        s.set_timeout(timeout)
        for c in constraints:
            s.add(c)
        for e in minimize:
            s.minimize(e)
        for e in maximize:
            s.maximize(e)
        result = s.check()
        import z3
        if result == z3.sat:
            return s.model()
        if result == z3.unknown:
            log.debug("Timeout encountered while solving expression using z3")
        raise UnsatError
    if not z3bridge.available():
        raise SolverUnavailable("z3 is not installed; cannot decide this query")
    z3 = z3bridge._z3()
    s = z3.Optimize()
    s.set(timeout=timeout)
    memo: Dict[int, object] = {}
    for c in constraints:
        raw = getattr(c, "raw", c)
        s.add(z3bridge.to_z3(raw, memo) if isinstance(raw, N.Node) else raw)
    for e in minimize:
        raw = getattr(e, "raw", e)
        s.minimize(z3bridge.to_z3(raw, memo) if isinstance(raw, N.Node) else raw)
    for e in maximize:
        raw = getattr(e, "raw", e)
        s.maximize(z3bridge.to_z3(raw, memo) if isinstance(raw, N.Node) else raw)
    t0 = time.time()
    result = s.check()
    if stats.enabled:
        stats.query_count += 1
        stats.solver_time += time.time() - t0
    if result == z3.sat:
        return Model([s.model()])
    if result == z3.unknown:
        log.debug("Timeout encountered while solving expression using z3")
    raise UnsatError


def _wrap(z3_model, assignment, progs):
    if _stock_model is not None:
        return _stock_model([z3_model])
    return Model([z3_model], assignment, progs)


def _accept(constraints, assignment, progs, timeout_ms: int):
    """get_model's rule for a GPU witness (north_star: every witness is
    re-verified by z3 before a model is returned): whenever z3 is present —
    z3 ASTs as given, mirror DAG nodes through ``z3bridge.to_z3`` —
    substitute + simplify must give True and a genuine z3 model is returned.
    Without z3 the witness is returned as is (it was evaluated bit-exactly on
    the device).  None when z3 rejects it."""
    if z3bridge.available():
        memo: Dict[int, object] = {}
        raws = [getattr(c, "raw", c) for c in constraints]
        raws = [z3bridge.to_z3(r, memo) if isinstance(r, N.Node) else r for r in raws]
        if raws:
            with _Phase("verify"):
                m = z3bridge.verify(raws, assignment, timeout_ms)
            if m is None:
                stats.rejected += 1
                log.warning("GPU witness rejected by z3; falling back")
                return None
            return _wrap(m, assignment, progs)
    return Model(None, assignment, progs)


# Hand-over from batch_is_possible to get_model (bounded, oldest dropped):
# sets whose batched search found a witness (get_model then returns it
# without searching again) and sets it missed (get_model goes straight to z3).
_BATCH_MEMO = 1 << 14
_batch_witness: "Dict[tuple, tuple]" = {}
_gpu_missed: "Dict[tuple, bool]" = {}


def _remember(d: dict, key, value) -> None:
    try:
        d[key] = value
    except TypeError:                      # unhashable constraint: nothing to hand over
        return
    if len(d) > _BATCH_MEMO:
        d.pop(next(iter(d)))


def _take(d: dict, key):
    try:
        return d.pop(key, None)
    except TypeError:
        return None


# Engine initialisation failures are remembered: a machine without a usable
# GPU pays for the attempt once, then every query goes straight to z3.
_engine_failed: Optional[str] = None


def _engine_failure(e: EngineUnavailable, current: Optional[str]) -> Optional[str]:
    """What ``_engine_failed`` becomes after ``e``: a device's first context
    failing disables the GPU path; an extra context (slot > 0, a device
    listed twice in DEVICES) failing does not — that query falls back to z3,
    the repeat is dropped from DEVICES and the device's working contexts
    keep serving."""
    global DEVICES
    slot = getattr(e, "slot", 0)
    if slot == 0:
        return str(e)
    # keep the device's working contexts (slots 0 .. slot-1) only
    dev, kept, out = getattr(e, "device", 0), 0, []
    for d in DEVICES:
        if d == dev:
            if kept >= slot:
                continue
            kept += 1
        out.append(d)
    DEVICES = out
    return current


def _prefilter(key, constraints, timeout: int, enforce_execution_time: bool = False):
    """GPU path of get_model: a model, or None (miss / rejected witness).
    The witness check gets what is left of the execution time (``_deadline``)."""
    global _engine_failed
    hit = _take(_batch_witness, key)
    if hit is None:
        if _take(_gpu_missed, key) or _engine_failed is not None or not GPU_ENABLED:
            return None
        with _Phase("flatten"):
            nodes = _raw_nodes(constraints)
        stats.gpu_queries += 1
        t0 = time.perf_counter()
        try:
            hit = gpu_search(nodes, budget_ms=min(timeout, SEARCH_BUDGET_MS))
        except EngineUnavailable as e:
            _engine_failed = _engine_failure(e, _engine_failed)
            raise
        finally:
            stats.gpu_time += time.perf_counter() - t0
        if hit is None:
            return None
    if enforce_execution_time:
        timeout = min(timeout, time_handler.time_remaining() - 500)
        if timeout <= 0:                      # get_model's fallback raises UnsatError
            return None
    m = _accept(constraints, hit[0], hit[1], timeout)
    if m is not None:
        stats.gpu_hits += 1
    return m


@lru_cache(maxsize=2 ** 23)
def get_model(constraints, minimize=(), maximize=(), enforce_execution_time=True):
    key = constraints
    timeout = args.solver_timeout
    if enforce_execution_time:
        timeout = min(timeout, time_handler.time_remaining() - 500)
        if timeout <= 0:
            raise UnsatError
    for constraint in constraints:
        if type(constraint) == bool and not constraint:
            raise UnsatError
    constraints = [c for c in constraints if type(c) != bool]

    if not minimize and not maximize:
        try:
            m = _prefilter(key, constraints, timeout, enforce_execution_time)
            if m is not None:
                return m
        except Unsupported as e:
            stats.unsupported += 1
            log.debug("GPU pre-filter: unsupported (%s)", e)
        except Exception as e:  # noqa: BLE001 - any engine failure falls back to z3
            stats.errors += 1
            log.debug("GPU pre-filter failed (%s: %s); falling back to z3", type(e).__name__, e)
        stats.fallbacks += 1
    # the fallback gets the reference's own timeout (support/model.py:26-31),
    # not what the pre-filter left of it: a GPU miss must not turn a query z3
    # solves near its timeout into an ``unknown`` -> UnsatError prune.  Under
    # enforce_execution_time it is still capped by the execution time left
    # NOW (minus the reference's 500 ms), so the GPU phase cannot push the
    # analysis past --execution-timeout
    timeout = _deadline(timeout, enforce_execution_time)
    return _z3_check(constraints, minimize, maximize, timeout)


def _deadline(timeout: int, enforce_execution_time: bool) -> int:
    """``timeout`` capped by the execution time left at this moment minus
    500 ms (the reference's rule, support/model.py:26-31, re-applied after
    the GPU phase); <= 0 raises UnsatError exactly as at the entry."""
    if enforce_execution_time:
        timeout = min(timeout, time_handler.time_remaining() - 500)
        if timeout <= 0:
            raise UnsatError
    return timeout


def batch_is_possible(constraint_sets, enforce_execution_time=True) -> List[bool]:
    """``[c.is_possible for c in constraint_sets]`` with ONE batched GPU
    witness search over all the sets.

    Reference: ``Constraints.is_possible``
    (``mythril/laser/ethereum/state/constraints.py:26-35``: possible iff
    ``get_model(tuple(self))`` does not raise ``UnsatError``), called once per
    state by LASER's state filters (``mythril/laser/ethereum/svm.py:201-203``
    open states per transaction, ``:257-262`` new states per step).  Every set
    then goes through ``get_model`` itself — its cache, timeout arithmetic,
    Python-bool handling and z3 fallback — so the answers are the ones the
    per-state loop gives and UNSAT is only concluded by z3: a set with a GPU
    witness hands it to get_model (accepted by the same rule, no second
    search), a set the batch missed goes straight to z3."""
    global _engine_failed
    sets = [tuple(c) for c in constraint_sets]
    timeout = args.solver_timeout
    if enforce_execution_time:
        timeout = min(timeout, time_handler.time_remaining() - 500)
    pending = []                          # (set, bucket programs)
    if timeout > 0 and _engine_failed is None and GPU_ENABLED:
        for cs in sets:
            if any(type(c) == bool and not c for c in cs):
                continue                                   # get_model raises UnsatError
            try:
                with _Phase("flatten"):
                    nodes = _raw_nodes([c for c in cs if type(c) != bool])
                buckets = dependence_buckets(nodes)
                with _Phase("refute"):
                    dead = _refuted_group(buckets, [_group_key(b) for b in buckets])
                if dead is not None:
                    # refuted on the host: get_model below sends it to z3
                    # without a search (the memo answers it)
                    stats.refuted += 1
                    _note_miss(dead, GROUND_MISS)
                    _remember(_gpu_missed, cs, True)
                    continue
                with _Phase("compile"):
                    progs = [_compile_search(b) for b in buckets]
            except Unsupported as e:
                stats.unsupported += 1
                log.debug("GPU pre-filter: unsupported (%s)", e)
                continue
            except Exception as e:  # noqa: BLE001
                stats.errors += 1
                log.debug("GPU pre-filter failed on a set: %s", e)
                continue
            pending.append((cs, progs))
    if pending:
        try:
            t0 = time.perf_counter()
            flat = [p for _, progs in pending for p in progs]
            n_cand = _n_cand(flat, min(timeout, SEARCH_BUDGET_MS))
            kinds: List[str] = []
            hits = iter(_search_sets([progs for _, progs in pending], n_cand, kinds))
            kinds_it = iter(kinds)
            stats.gpu_time += time.perf_counter() - t0
            for cs, progs in pending:
                found = [next(hits) for _ in progs]
                how = [next(kinds_it) for _ in progs]
                stats.gpu_queries += 1
                stats.gpu_candidates += sum(n_cand if k < 0 else k + 1
                                            for (k, _), h in zip(found, how) if h == SEARCHED)
                for p, (k, _), h in zip(progs, found, how):
                    # only a group that was launched (or folded to false)
                    # missed; a group skipped for a false sibling was not
                    # searched, and its key must not block later queries
                    if k < 0 and p.group_key is not None and h in (SEARCHED, GROUND_FALSE):
                        _note_miss(p.group_key, GROUND_MISS if h == GROUND_FALSE else n_cand)
                if any(k < 0 for k, _ in found):
                    # the set goes straight to z3 only when the batch searched
                    # it as far as get_model alone would have; otherwise
                    # get_model runs its own (budgeted) search
                    if n_cand >= _n_cand(progs, min(timeout, SEARCH_BUDGET_MS)):
                        _remember(_gpu_missed, cs, True)
                else:
                    a = _merge([w for _, w in found])
                    _remember(_batch_witness, cs, (a, progs))
        except EngineUnavailable as e:
            _engine_failed = _engine_failure(e, _engine_failed)
            log.debug("GPU pre-filter unavailable: %s", e)
        except Exception as e:  # noqa: BLE001
            stats.errors += 1
            log.debug("GPU pre-filter failed (%s: %s)", type(e).__name__, e)
    results = []
    for cs in sets:
        try:
            # the call form of Constraints.is_possible (constraints.py:32), so
            # the lru_cache entry is the one the per-state loop would hit
            if enforce_execution_time:
                get_model(cs)
            else:
                get_model(cs, enforce_execution_time=False)
            results.append(True)
        except UnsatError:
            results.append(False)
    return results


def filter_possible(states, constraints_of=lambda s: s.world_state.constraints):
    """Drop-in for LASER's state filters
    ``[s for s in states if s.world_state.constraints.is_possible]``
    (``svm.py:257-262``; ``svm.py:201-203`` passes
    ``constraints_of=lambda s: s.constraints``), one batched search."""
    states = list(states)
    keep = batch_is_possible([constraints_of(s) for s in states])
    return [s for s, k in zip(states, keep) if k]


def _patch_statistics(cls) -> None:
    """Mythril's ``SolverStatistics`` (a singleton, logged by ``fire_lasers``
    at ``mythril_analyzer.py:181``) prints the pre-filter's counters after
    its own two lines."""
    if getattr(cls, "_mythril_amd_patched", False):
        return
    base = cls.__repr__

    def __repr__(self):
        return base(self) + "\n" + stats.gpu_report()
    cls.__repr__ = __repr__
    cls._mythril_amd_patched = True


def install() -> None:
    """Rebind ``get_model`` in a Mythril installation: the three names bound
    by ``from ... import get_model``, and share Mythril's
    ``args`` / ``time_handler`` singletons, its ``Optimize`` wrapper, its
    ``Model`` class and its ``SolverStatistics``."""
    import importlib
    global args, time_handler, _stock_optimize, _stock_model
    configure_from_env()
    args = importlib.import_module("mythril.support.support_args").args
    time_handler = importlib.import_module("mythril.laser.ethereum.time_handler").time_handler
    smt = importlib.import_module("mythril.laser.smt")
    _stock_optimize = smt.Optimize
    _stock_model = smt.Model
    _patch_statistics(importlib.import_module(
        "mythril.laser.smt.solver.solver_statistics").SolverStatistics)
    get_model.cache_clear()
    for mod in ("mythril.support.model", "mythril.analysis.solver",
                "mythril.laser.ethereum.state.constraints"):
        m = importlib.import_module(mod)
        m.get_model = get_model
    # concrete hashes of reported transactions: one GPU Keccak batch
    # (analysis/solver.py:119-152 -> mythril_amd.sha)
    solver = importlib.import_module("mythril.analysis.solver")
    if hasattr(solver, "_replace_with_actual_sha"):
        from .sha import replace_with_actual_sha
        kfm = importlib.import_module("mythril.laser.ethereum.keccak_function_manager")
        sf = smt.symbol_factory

        def _replace(concrete_transactions, model, code=None):
            replace_with_actual_sha(concrete_transactions, model,
                                    kfm.keccak_function_manager, code, symbol_factory=sf)
        solver._replace_with_actual_sha = _replace
