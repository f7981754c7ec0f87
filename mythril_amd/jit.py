"""Compiled programs: the batch path without interpretive dispatch
(DESIGN.md §3.5).

The assembly interpreter (asmgen.py) spends, per IR record, a record
prefetch, a computed jump (``s_setpc``: an instruction-fetch redirect) and
GPR-index mode switches around every register-file access.  For a batch that
evaluates each program under 2^20 candidates that cost is paid 2^20 / 64
times per record, so the batch path compiles each program instead:

* every record is rendered by the SAME handler generator the interpreter is
  built from (``asmgen.emit_handler`` with ``asmgen.JIT`` set: no prefetch,
  no dispatch), then **specialised** to the record: GPR-index mode is
  resolved statically (each indexed VGPR operand becomes the register the
  index selected), record fields become immediates or are folded through the
  scalar arithmetic that consumes them, branches on them are decided, and the
  mode switches disappear;
* the records of a program are laid out as one straight line (out-of-line
  blocks collected and placed every few records behind a jump), ending in a
  return to the interpreter kernel, which calls the program's code through
  the ``jit_entry`` of its descriptor (``mg_pdesc``, one ``s_swappc``);
* division and ``bvumul_noovfl`` stay shared bodies (hundreds of VALU each):
  the call sets the record fields they read and ``s_swappc``s to them.

The interpreter stays the path for single ``get_model`` queries (a few ms of
host compile here would cost more than the dispatch it saves).  Programs are
assembled with the ROCm LLVM assembler and linked into a code object next to
a tiny stub kernel (``lib/mg_jit_stub.s``, built from csrc/mg_jit_stub.hip);
``mg_jit_attach`` loads it and points the descriptors at the code.
Correctness is checked on the CPU by running the generated text through the
instruction-level simulator (tests/asm_sim.py), and on the GPU by the same
parity tests as the interpreter (tests/test_gpu_bench_parity.py).
"""

from __future__ import annotations

import functools
import os
import re
import subprocess
import tempfile
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import asmgen as G
from . import irdefs as I

LLVM_BIN = os.environ.get("MYTHGPU_LLVM_BIN", "/opt/rocm/lib/llvm/bin")
ARCH = os.environ.get("MYTHGPU_ARCH", "gfx950")
LIBDIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
STUB = os.path.join(LIBDIR, "mg_jit_stub.s")
M32 = 0xFFFFFFFF
BANK0 = G.BANK[0]
COLD_FLUSH = 32            # out-of-line blocks are placed every this many records
BODY_LABEL = {"DIV": ".Lbody_DIV_jb", "UMULNO": ".Lbody_UMULNO_jb"}


class JitUnsupported(Exception):
    """A record the specialiser cannot resolve statically (the program then
    stays on the interpreter)."""


# ---------------------------------------------------------------------------
# templates: handler text rendered in JIT mode
# ---------------------------------------------------------------------------

_TEMPLATES: Dict[Tuple[str, int], List[str]] = {}


def _render(fn) -> List[str]:
    G.JIT = True
    try:
        a = G.Asm()
        fn(a)
        a.flush_cold()
        return list(a.lines)
    finally:
        G.JIT = False


def template(name: str, var: int) -> List[str]:
    key = (name, var)
    t = _TEMPLATES.get(key)
    if t is None:
        t = _render(lambda a: G.emit_handler(a, name, var, 0))
        _TEMPLATES[key] = t
    return t


def bodies() -> List[str]:
    """The shared heavy bodies in JIT form: no record prefetch, and the
    dispatch replaced by a return through s[JIT_BODY_RET] (with GPR-index
    mode off: the straight-line code after the call is not indexed)."""
    out = []
    # one Asm for both: its label counter keeps their labels distinct
    for line in _render(lambda a: (G.body_umulno(a), G.body_div(a))):
        if line == "@@END":
            out.append("    s_setpc_b64 %s" % G.sp(G.JIT_BODY_RET))
        else:
            out.append(line)
    labels = [l for l in out if l.endswith(":")]
    assert len(labels) == len(set(labels)), "duplicate labels in the JIT bodies"
    return [_subst(l, "jb") for l in out]


def _subst(line: str, tag: str) -> str:
    line = line.replace("%=", tag)
    if "%[" in line:
        for k, r in G.PINNED.items():
            line = line.replace("%%[%s]" % k, r)
    return line


# ---------------------------------------------------------------------------
# instruction text
# ---------------------------------------------------------------------------

def _tokens(rest: str) -> Tuple[List[str], List[str]]:
    """Operands (split at depth-0 commas) and trailing modifiers
    (``offset:16``, ``clamp``, ``op_sel:[1,0]``) of an instruction."""
    ops, mods, cur, depth = [], [], "", 0
    for ch in rest:
        if ch in "([":
            depth += 1
        elif ch in ")]":
            depth -= 1
        if ch == "," and depth == 0:
            ops.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        ops.append(cur.strip())
    if ops:
        last = ops[-1]
        # modifiers follow the last operand after whitespace (not inside ( ))
        depth, cut = 0, None
        for i, ch in enumerate(last):
            if ch in "([":
                depth += 1
            elif ch in ")]":
                depth -= 1
            elif ch == " " and depth == 0:
                cut = i
                break
        if cut is not None:
            mods = last[cut:].split()
            ops[-1] = last[:cut].strip()
    return ops, mods


@functools.lru_cache(maxsize=1 << 18)
def _parse_cached(t: str):
    parts = t.split(None, 1)
    ops, mods = _tokens(parts[1]) if len(parts) > 1 else ([], [])
    return parts[0], tuple(ops), tuple(mods)


def parse(line: str):
    m, ops, mods = _parse_cached(line.strip())
    return m, list(ops), list(mods)


def render(m: str, ops: Sequence[str], mods: Sequence[str] = ()) -> str:
    s = "    " + m
    if ops:
        s += " " + ", ".join(ops)
    if mods:
        s += " " + " ".join(mods)
    return s


_VREG = re.compile(r"(-?)v(\d+)$")
_VPAIR = re.compile(r"(-?)v\[(\d+):(\d+)\]$")
_SREG = re.compile(r"s(\d+)$")
_SPAIR = re.compile(r"s\[(\d+):(\d+)\]$")


@functools.lru_cache(maxsize=1 << 16)
def vreg(tok: str) -> Optional[Tuple[int, int]]:
    m = _VREG.match(tok)
    if m:
        return int(m.group(2)), 1
    m = _VPAIR.match(tok)
    if m:
        return int(m.group(2)), int(m.group(3)) - int(m.group(2)) + 1
    return None


@functools.lru_cache(maxsize=1 << 16)
def sreg(tok: str) -> Optional[Tuple[int, int]]:
    m = _SREG.match(tok)
    if m:
        return int(m.group(1)), 1
    m = _SPAIR.match(tok)
    if m:
        return int(m.group(1)), int(m.group(2)) - int(m.group(1)) + 1
    return None


def shift_vreg(tok: str, off: int) -> str:
    m = _VREG.match(tok)
    if m:
        return "%sv%d" % (m.group(1), int(m.group(2)) + off)
    m = _VPAIR.match(tok)
    if m:
        return "%sv[%d:%d]" % (m.group(1), int(m.group(2)) + off, int(m.group(3)) + off)
    return tok


def int_value(tok: str) -> Optional[int]:
    try:
        return int(tok, 0) & M32
    except ValueError:
        return None


@functools.lru_cache(maxsize=4096)
def n_dest(m: str) -> int:
    if m.startswith("v_cmp"):
        return 1
    if re.match(r"v_(add|sub|subrev|addc|subb|subbrev)_co_u32", m) or \
            m.startswith(("v_mad_u64_u32", "v_mad_i64_i32")):
        return 2
    if m.startswith("v_"):
        return 1
    if m.startswith(("global_store", "scratch_store", "ds_write", "buffer_store")):
        return 0
    if m.startswith(("global_load", "scratch_load", "ds_read", "buffer_load", "s_load")):
        return 1
    if m.startswith(("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_waitcnt", "s_nop",
                     "s_setpc", "s_endpgm", "s_set_gpr_idx", "s_swappc")):
        return 0
    return 1


def is_salu(m: str) -> bool:
    return m.startswith("s_") and not m.startswith(("s_load", "s_waitcnt", "s_nop", "s_branch",
                                                     "s_cbranch", "s_setpc", "s_swappc",
                                                     "s_getpc", "s_endpgm", "s_set_gpr_idx"))


def _inline(v: int) -> Optional[str]:
    """The value as an inline constant, when it is one (-16..64)."""
    x = v - (1 << 32) if v >> 31 else v
    return str(x) if -16 <= x <= 64 else None


# scalar ops folded when every input is known: value, scc
def _fold(m: str, vals: List[int]) -> Optional[Tuple[int, Optional[int]]]:
    a = vals[0] if vals else 0
    b = vals[1] if len(vals) > 1 else 0
    if m == "s_mov_b32":
        return a, None
    if m == "s_movk_i32":
        x = a & 0xFFFF
        return (x - 0x10000 if x & 0x8000 else x) & M32, None
    if m == "s_add_u32":
        r = a + b
        return r & M32, int(r >> 32 != 0)
    if m == "s_sub_u32":
        return (a - b) & M32, int(b > a)
    if m in ("s_and_b32", "s_or_b32", "s_xor_b32"):
        r = {"s_and_b32": a & b, "s_or_b32": a | b, "s_xor_b32": a ^ b}[m]
        return r, int(r != 0)
    if m == "s_lshl_b32":
        r = (a << (b & 31)) & M32
        return r, int(r != 0)
    if m == "s_lshr_b32":
        r = a >> (b & 31)
        return r, int(r != 0)
    if m == "s_bfe_u32":
        off, width = b & 31, (b >> 16) & 0x7F
        r = (a >> off) & ((1 << width) - 1)
        return r, int(r != 0)
    if m == "s_mul_i32":
        return (a * b) & M32, None
    return None


_CMP = {"s_cmp_eq_u32": lambda a, b: a == b, "s_cmp_lg_u32": lambda a, b: a != b,
        "s_cmp_lt_u32": lambda a, b: a < b, "s_cmp_le_u32": lambda a, b: a <= b,
        "s_cmp_gt_u32": lambda a, b: a > b, "s_cmp_ge_u32": lambda a, b: a >= b,
        "s_bitcmp1_b32": lambda a, b: (a >> (b & 31)) & 1 == 1}


# ---------------------------------------------------------------------------
# the specialiser
# ---------------------------------------------------------------------------

RECORD_SGPRS = frozenset(range(BANK0, BANK0 + 8))
# memos of a template's analysis, keyed by the template list's id() and
# holding the list itself: a hit must be that very list (a layout switch
# drops the templates, and a new list may reuse a dropped one's id)
_TARGETS: Dict[int, tuple] = {}


def _branch_targets(lines: Sequence[str]) -> frozenset:
    """Labels some branch of the template jumps to (the others are only
    fall-through points: no join, no state reset)."""
    key = id(lines)
    hit = _TARGETS.get(key)
    if hit is None or hit[0] is not lines:
        out = set()
        for l in lines:
            t = l.strip()
            if t.startswith(("s_branch", "s_cbranch")):
                out.add(t.split()[1])
        hit = _TARGETS[key] = (lines, frozenset(out))
    return hit[1]


_REACH: Dict[int, object] = {}


def _reach_reads(lines: Sequence[str]):
    """(R, at): R[i] = the SGPRs some line on a control-flow path from line
    i reads (i included; later writes ignored, so an over-approximation of
    liveness, but along the template's branches and fall-throughs rather
    than its text order); at: label -> line index.  A branch materializes
    only what its target may read, so a value the fall-through path uses
    as a literal stays unmaterialized there."""
    key = id(lines)
    hit = _REACH.get(key)
    if hit is not None and hit[0] is lines:
        return hit[1]
    n = len(lines)
    uses: List[frozenset] = []
    succ: List[Tuple[int, ...]] = []
    at: Dict[str, int] = {}
    parsed = []
    for i, l in enumerate(lines):
        t = _subst(l.strip(), "x")
        parsed.append(t)
        if t.endswith(":"):
            at[t[:-1]] = i
    for i, t in enumerate(parsed):
        nxt = (i + 1,) if i + 1 < n else ()
        if not t or t.endswith(":"):
            uses.append(frozenset())
            succ.append(nxt)
            continue
        if t.startswith("@@"):
            uses.append(frozenset())
            succ.append(())                      # END / HALT / CALL: no fall-through
            continue
        m, ops, _ = parse(t)
        u = set()
        for x in ops[n_dest(m):] if not m.startswith(("s_set_gpr_idx", "s_cmp", "s_bitcmp")) else ops:
            r = sreg(x)
            if r:
                u.update(range(r[0], r[0] + r[1]))
        uses.append(frozenset(u))
        if m == "s_branch":
            succ.append((at[ops[0]],) if ops[0] in at else ())
        elif m.startswith("s_cbranch"):
            succ.append(nxt + ((at[ops[0]],) if ops[0] in at else ()))
        elif m.startswith(("s_setpc", "s_endpgm")):
            succ.append(())
        else:
            succ.append(nxt)
    R = [set(u) for u in uses]
    changed = True
    while changed:
        changed = False
        for i in range(n - 1, -1, -1):
            acc = R[i]
            k = len(acc)
            for j in succ[i]:
                acc |= R[j]
            if len(acc) != k:
                changed = True
    out = ([frozenset(r) for r in R], at)
    _REACH[key] = (lines, out)
    return out


class _State:
    def __init__(self, rec: Sequence[int]):
        self.rec = {BANK0 + k: int(rec[k]) & M32 for k in range(8)}
        self.known: Dict[int, int] = dict(self.rec)
        self.mat: set = set()           # known SGPRs whose register holds the value
        self.idx: Optional[Tuple[int, frozenset]] = None
        self.scc: Optional[int] = None


def specialize(lines: Sequence[str], rec: Sequence[int], tag: str):
    """(hot lines, cold lines, heavy body called or None) of one record:
    ``lines`` is the handler's JIT template, ``rec`` its 8 record words.

    Scalar state: the record fields (s40..s47, never written by a handler)
    are known on every path.  Values derived from them by folded scalar
    arithmetic are known along the straight path; before any branch or join
    the live ones are materialized (``s_mov_b32``) so the register holds
    them on every path, and after a label only the record fields are known.
    GPR-index state must agree on every path into a label (checked)."""
    st = _State(rec)
    reach, _ = _reach_reads(lines)
    label_at = {}                        # label (this record's name) -> template line
    for k, raw in enumerate(lines):
        t = raw.strip()
        if t.endswith(":"):
            label_at[_subst(t[:-1], tag)] = k
    targets = {l.replace("%=", tag) for l in _branch_targets(lines)}
    hot: List[str] = []
    cold: List[str] = []
    out = hot
    idx_in: Dict[str, object] = {}       # label -> index state on the branches into it
    idx_at: Dict[str, object] = {}       # label -> index state where it was placed
    call = None
    fallthrough = True
    dead = False                         # after a branch folded taken: skip to a reached label
    dead_labels = set()                  # labels skipped in such code (no branch may go there)

    def emit(text):
        out.append(text)

    def materialize(regs):
        for r in regs:
            if r in st.known and r not in st.mat:
                emit("    s_mov_b32 s%d, 0x%x" % (r, st.known[r]))
                st.mat.add(r)

    def settle(label):
        """Before a branch to / a fall-through into ``label``: derived values
        the code from there may read go into their registers."""
        j = label_at.get(label)
        need = reach[j] if j is not None else None
        materialize(sorted(r for r in st.known if r not in RECORD_SGPRS and
                           (need is None or r in need)))

    def written(regs):
        for r in regs:
            st.known.pop(r, None)
            st.mat.discard(r)

    def sregs_of(tok):
        r = sreg(tok)
        return list(range(r[0], r[0] + r[1])) if r else []

    def branch_to(label):
        if label in dead_labels:
            raise JitUnsupported("branch to %s in code a folded branch skipped" % label)
        if label in idx_at:
            if idx_at[label] != st.idx:
                raise JitUnsupported("index state differs on a branch back to %s" % label)
        elif label in idx_in:
            if idx_in[label] != st.idx:
                raise JitUnsupported("index state differs on the branches into %s" % label)
        else:
            idx_in[label] = st.idx

    for i, raw in enumerate(lines):
        line = _subst(raw, tag)
        if "@F" in line:            # a record field as an instruction immediate
            line = re.sub(r"@F(\d)(?:\+(\d+))?@",
                          lambda mm: str((int(rec[int(mm.group(1))]) + int(mm.group(2) or 0))
                                         & M32), line)
        t = line.strip()
        if not t:
            continue
        if t == "@@END":
            out = cold
            fallthrough = False
            continue
        # code a folded-taken branch skipped (up to a label a kept branch
        # reaches): nothing in it is emitted or changes the index state —
        # only where later lines go (@@HALT / @@CALL end a hot block) is kept
        skipped = dead and not fallthrough
        if t == "@@HALT":
            if not skipped:
                emit("    s_setpc_b64 %s" % G.sp(G.JIT_RET))
            out = cold
            fallthrough = False
            continue
        if t.startswith("@@CALL"):
            if skipped:
                out = cold
                continue
            _, body, bits = t.split()
            kind = "DIV" if "DIV" in body else "UMULNO"
            # the body reads its record from S_CUR and its variant from S_VAR
            for k in (G.F_D, G.F_A, G.F_B, G.F_W, G.F_MOFF):
                emit("    s_mov_b32 s%d, 0x%x" % (G.S_CUR + k, int(rec[k]) & M32))
            emit("    s_mov_b32 s%d, 0x%x" % (G.S_VAR, int(bits)))
            lab = ".Lcall_%s" % tag
            emit("    s_getpc_b64 %s" % G.sp(G.S_JMP))
            emit(lab + ":")
            emit("    s_add_u32 s%d, s%d, (%s - %s)" % (G.S_JMP, G.S_JMP, BODY_LABEL[kind], lab))
            emit("    s_addc_u32 s%d, s%d, 0" % (G.S_JMP + 1, G.S_JMP + 1))
            emit("    s_swappc_b64 %s, %s" % (G.sp(G.JIT_BODY_RET), G.sp(G.S_JMP)))
            call = kind
            out = cold
            fallthrough = False
            continue
        if t.endswith(":"):
            lab = t[:-1]
            if lab not in targets:
                if dead:
                    continue
                if not fallthrough:
                    raise JitUnsupported("label %s is never reached" % lab)
                continue                     # no branch comes here: not a join
            if dead and lab not in idx_in:
                dead_labels.add(lab)         # only branches from skipped code come here
                continue
            dead = False
            incoming = idx_in.pop(lab, "none")
            if fallthrough:
                settle(lab)
                if incoming != "none" and incoming != st.idx:
                    raise JitUnsupported("index state differs at label %s" % lab)
            elif incoming != "none":
                st.idx = incoming
            else:
                raise JitUnsupported("label %s reached only from later code" % lab)
            idx_at[lab] = st.idx
            st.known = dict(st.rec)
            st.mat = set()
            st.scc = None
            fallthrough = True
            emit(t)
            continue
        m, ops, mods = parse(t)
        if skipped:
            continue                         # the folded branch's skipped code
        # ---- GPR-index mode: resolved statically ----------------------------
        if m == "s_set_gpr_idx_on":
            r = sreg(ops[0])
            if r is None or r[0] not in st.known:
                raise JitUnsupported("dynamic GPR index")
            modes = frozenset(re.search(r"gpr_idx\(([^)]*)\)", ops[1]).group(1).split(","))
            st.idx = (st.known[r[0]] & 0xFF, modes)
            continue
        if m == "s_set_gpr_idx_idx":
            r = sreg(ops[0])
            if r is None or r[0] not in st.known or st.idx is None:
                raise JitUnsupported("dynamic GPR index")
            st.idx = (st.known[r[0]] & 0xFF, st.idx[1])
            continue
        if m == "s_set_gpr_idx_mode":
            if st.idx is None:
                raise JitUnsupported("index mode change while off")
            st.idx = (st.idx[0], frozenset(re.search(r"gpr_idx\(([^)]*)\)", ops[0]).group(1).split(",")))
            continue
        if m == "s_set_gpr_idx_off":
            st.idx = None
            continue
        if not fallthrough:
            if dead:
                continue                     # the folded branch's skipped code
            raise JitUnsupported("unreachable code after a jump: %s" % t)
        # ---- control flow ------------------------------------------------
        if m in ("s_cbranch_scc0", "s_cbranch_scc1") and st.scc is not None:
            if st.scc == (1 if m == "s_cbranch_scc1" else 0):
                settle(ops[0])
                branch_to(ops[0])
                emit(render("s_branch", ops))
                fallthrough, dead = False, True
            continue
        if m.startswith("s_cbranch") or m == "s_branch":
            settle(ops[0])
            branch_to(ops[0])
            emit(render(m, ops, mods))
            if m == "s_branch":
                fallthrough = False
            continue
        nd = n_dest(m)
        # ---- scalar ALU: fold known inputs -------------------------------
        if is_salu(m):
            dst, srcs = ops[:nd], ops[nd:]
            if m in _CMP:
                vals = [st.known.get(sreg(x)[0]) if sreg(x) and sreg(x)[1] == 1 else
                        (int_value(x) if not sreg(x) else None) for x in srcs]
                if all(v is not None for v in vals):
                    st.scc = int(_CMP[m](vals[0], vals[1]))
                    continue
            if m == "s_cselect_b64" and st.scc is not None:
                m, srcs = "s_mov_b64", [srcs[0] if st.scc else srcs[1]]
                if srcs[0] == dst[0]:
                    continue                 # keeps its value
            if m == "s_mov_b64":
                rs, dr = sregs_of(srcs[0]), sregs_of(dst[0])
                if dr and rs and all(r in st.known for r in rs):
                    vals = [st.known[r] for r in rs]
                    written(dr)
                    for d_, v_ in zip(dr, vals):
                        st.known[d_] = v_
                    continue
                if dr and not rs and int_value(srcs[0]) == 0:
                    written(dr)
                    for d_ in dr:
                        st.known[d_] = 0
                    continue
            one_reg = all((sreg(x) is None or sreg(x)[1] == 1) for x in srcs)
            vals = [st.known.get(sreg(x)[0]) if sreg(x) else int_value(x) for x in srcs]
            if one_reg and dst and sreg(dst[0]) and sreg(dst[0])[1] == 1 and \
                    all(v is not None for v in vals):
                r = _fold(m, vals)
                if r is not None:
                    d_ = sreg(dst[0])[0]
                    written([d_])
                    st.known[d_] = r[0]
                    if r[1] is not None:
                        st.scc = r[1]
                    continue
            # runtime: a known register input becomes a literal (one per
            # instruction), the others are materialized
            lit = sum(1 for x in srcs if not sreg(x) and int_value(x) is not None and
                      _inline(int_value(x)) is None and not x.startswith("("))
            new_srcs = []
            for x in srcs:
                r = sreg(x)
                if r and r[1] == 1 and r[0] in st.known and r[0] not in st.mat:
                    v = st.known[r[0]]
                    if _inline(v) is not None:
                        new_srcs.append(_inline(v))
                        continue
                    if lit == 0:
                        new_srcs.append("0x%x" % v)
                        lit = 1
                        continue
                if r:
                    materialize(range(r[0], r[0] + r[1]))
                new_srcs.append(x)
            emit(render(m, dst + new_srcs, mods))
            for x in dst:
                written(sregs_of(x))
            st.scc = None
            continue
        # ---- scalar memory: a known offset becomes the immediate ----------
        if m.startswith("s_load"):
            r = sreg(ops[2]) if len(ops) > 2 else None
            if r and r[1] == 1 and r[0] in st.known and st.known[r[0]] < (1 << 20):
                ops = ops[:2] + ["0x%x" % st.known[r[0]]]
            else:
                for x in ops[1:]:
                    materialize(sregs_of(x))
            emit(render(m, ops, mods))
            written(sregs_of(ops[0]))
            continue
        # ---- vector ALU: static GPR indexing, known scalar inputs ---------
        if m.startswith("v_"):
            new = []
            for k, x in enumerate(ops):
                pos = "DST" if k < nd else ("SRC%d" % (k - nd) if k - nd < 3 else None)
                if st.idx is not None and pos in st.idx[1] and vreg(x):
                    x = shift_vreg(x, st.idx[0])
                if k >= nd:
                    r = sreg(x)
                    if r and any(q in st.known and q not in st.mat for q in range(r[0], r[0] + r[1])):
                        if r[1] == 1 and _inline(st.known[r[0]]) is not None:
                            x = _inline(st.known[r[0]])
                        else:
                            materialize(range(r[0], r[0] + r[1]))
                new.append(x)
            for x in new:
                vr = vreg(x)
                if vr and vr[0] + vr[1] > G.NVGPR_KERNEL:
                    raise JitUnsupported("VGPR v%d outside the kernel's budget" % (vr[0] + vr[1] - 1))
            emit(render(m, new, mods))
            for x in new[:nd]:
                written(sregs_of(x))
            continue
        # ---- everything else (vector memory, LDS, waits, getpc) -----------
        for x in ops[nd:]:
            materialize(sregs_of(x))
        emit(render(m, ops, mods))
        for x in ops[:nd]:
            written(sregs_of(x))
    if idx_in:
        raise JitUnsupported("branches to labels outside the handler: %s" % sorted(idx_in))
    return hot, cold, call


# ---------------------------------------------------------------------------
# copy coalescing: the interpreter stages operands in temporaries (Y <- slot,
# R = op(...), slot <- R) because its register file is indexed; with fixed
# registers the staging copies can go
# ---------------------------------------------------------------------------

SLOTS = range(G.FB, G.FB + 8 * G.NREG)                 # v8..v135
TEMPS = frozenset(list(range(G.XB, G.XB + 8)) + list(range(G.YB, G.TB + G.NT)))


@functools.lru_cache(maxsize=1 << 16)
def _vregs_t(tok: str) -> Tuple[int, ...]:
    r = vreg(tok)
    return tuple(range(r[0], r[0] + r[1])) if r else ()


def _vregs(tok: str) -> List[int]:
    return list(_vregs_t(tok))


class _Ins:
    """One instruction of a straight segment: VGPR defs / uses per operand."""
    __slots__ = ("m", "ops", "mods", "nd", "masked", "load", "valu")

    def __init__(self, m, ops, mods, masked):
        self.m, self.ops, self.mods, self.masked = m, ops, mods, masked
        self.nd = n_dest(m)
        self.load = m.startswith(("global_load", "scratch_load", "ds_read", "buffer_load"))
        self.valu = m.startswith("v_")

    def def_ops(self):
        return [i for i in range(self.nd) if _vregs_t(self.ops[i])]

    def use_ops(self):
        return [i for i in range(self.nd, len(self.ops)) if _vregs_t(self.ops[i])]

    def defs(self):
        out = set()
        for i in range(self.nd):
            out.update(_vregs_t(self.ops[i]))
        return out

    def uses(self):
        out = set()
        for i in range(self.nd, len(self.ops)):
            out.update(_vregs_t(self.ops[i]))
        if self.masked:                 # inactive lanes keep the old value
            for i in range(self.nd):
                out.update(_vregs_t(self.ops[i]))
        return out

    def text(self):
        return render(self.m, self.ops, self.mods)


def _rename(tok: str, mp: Dict[int, int]) -> Optional[str]:
    """tok with its registers mapped (all or none, contiguously), or None."""
    regs = _vregs(tok)
    if not regs or not any(r in mp for r in regs):
        return tok
    if not all(r in mp for r in regs):
        return None
    new = [mp[r] for r in regs]
    if new != list(range(new[0], new[0] + len(new))) or (len(new) > 1 and new[0] % 2):
        return None
    return shift_vreg(tok, new[0] - regs[0])


def _copy(ins: _Ins) -> Optional[Tuple[List[int], List[int]]]:
    if ins.m not in ("v_mov_b32", "v_mov_b64") or ins.mods or len(ins.ops) != 2:
        return None
    d, s_ = _vregs(ins.ops[0]), _vregs(ins.ops[1])
    if not d or not s_ or len(d) != len(s_) or ins.ops[1].startswith("-"):
        return None
    return d, s_


def _forward(seg: List[Optional[_Ins]], final: bool) -> None:
    """temp <- slot copies: later reads of the temp read the slot instead;
    the copy goes when no read of the temp needs it any more."""
    for k, ins in enumerate(seg):
        c = _copy(ins) if ins is not None else None
        if c is None or ins.masked:
            continue                        # a masked copy merges: the temp != the slot
        d, s_ = c
        if not all(r in TEMPS for r in d) or not all(r in SLOTS for r in s_):
            continue
        mp = dict(zip(d, s_))
        state = {t: "active" for t in d}    # active: substitutable; stale: slot changed
        keep = False
        for j in range(k + 1, len(seg)):
            x = seg[j]
            if x is None:
                continue
            for i in x.use_ops():
                regs = [r for r in _vregs(x.ops[i]) if state.get(r) in ("active", "stale")]
                if not regs:
                    continue
                live = {t: mp[t] for t in d if state[t] == "active"}
                t = _rename(x.ops[i], live)
                if t is None:
                    keep = True
                else:
                    x.ops[i] = t
            dd = x.defs()
            if x.masked and any(state.get(r) in ("active", "stale") for r in dd):
                keep = True                 # inactive lanes keep the temp's value
            for r in dd:
                if state.get(r) in ("active", "stale"):
                    state[r] = "dead"       # rewritten: later reads are not ours
            for t in d:
                if state[t] == "active" and mp[t] in dd:
                    state[t] = "stale"      # the slot changed under the temp
        if not final and any(v != "dead" for v in state.values()):
            keep = True                     # may be read after the segment
        if not keep:
            seg[k] = None


def _read_later(seg, start, reg) -> bool:
    for x in seg[start:]:
        if x is None:
            continue
        if reg in x.uses():
            return True
        if reg in x.defs():
            return False
    return False


def _backward(seg: List[Optional[_Ins]], final: bool) -> None:
    """slot <- temp copies: the instructions that build the temp write the
    slot directly; the copy goes."""
    for k in range(len(seg) - 1, -1, -1):
        ins = seg[k]
        c = _copy(ins) if ins is not None else None
        if c is None or ins.masked:
            continue
        d, s_ = c
        if not all(r in SLOTS for r in d) or not all(r in TEMPS for r in s_):
            continue
        mp = dict(zip(s_, d))               # temp -> slot
        # the temp must be dead after the copy
        dead = True
        for r in s_:
            if _read_later(seg, k + 1, r):
                dead = False
            elif not final and not any(r in x.defs() for x in seg[k + 1:] if x is not None):
                dead = False
        if not dead:
            continue
        need = set(s_)                      # temps whose full definition is still ahead (backward)
        web = []
        ok = False
        for j in range(k - 1, -1, -1):
            x = seg[j]
            if x is None:
                continue
            touched = (x.defs() | x.uses()) & set(d)
            if touched:
                break                        # the slot is read / written inside the web
            dd = x.defs() & set(mp)
            uu = x.uses() & set(mp)
            if not dd and not uu:
                continue
            if dd and (x.load or not x.valu):
                break
            web.append(j)
            for r in dd & need:
                if not x.masked and r not in x.uses():
                    need.discard(r)         # a full definition: the web starts here
            if not need:
                ok = True
                break
        if not ok:
            continue
        # rename every operand of the web (all-or-nothing per operand)
        new_ops = {}
        for j in web:
            x = seg[j]
            ops = list(x.ops)
            for i in range(len(ops)):
                t = _rename(ops[i], mp)
                if t is None:
                    break
                ops[i] = t
            else:
                new_ops[j] = ops
                continue
            break
        else:
            for j, ops in new_ops.items():
                seg[j].ops = ops
            seg[k] = None


def coalesce(lines: List[str], final: bool = True) -> List[str]:
    """Drop the staging copies of one record's straight-line code.  Segments
    end at labels and branches (the analysis never crosses them);
    ``final``: the record's temporaries are dead at its end (true for every
    record: handlers never pass values in temporaries)."""
    out: List[str] = []
    seg: List[Optional[_Ins]] = []
    masked = False

    def flush(last: bool):
        _forward(seg, last)
        _backward(seg, last)
        out.extend(x.text() for x in seg if x is not None)
        seg.clear()

    for l in lines:
        t = l.strip()
        if t.endswith(":") or t.startswith(("s_branch", "s_cbranch", "s_setpc", "s_swappc",
                                            "s_getpc")):
            flush(False)
            out.append(l)
            continue
        m, ops, mods = parse(t)
        if m in ("s_and_saveexec_b64", "s_andn1_saveexec_b64") or \
                (m.startswith("s_") and ops[:1] == ["exec"] and m != "s_mov_b64"):
            masked = True
        elif m == "s_mov_b64" and ops[:1] == ["exec"]:
            masked = ops[1] == G.PINNED["active"]     # a restore, or the active lanes
        seg.append(_Ins(m, ops, mods, masked))
    flush(True)
    return out


# coalescing is memoised up to a relabelling of register-file slots: records
# that differ only in their slots (most cache misses above) give the same
# text once every 8-register file block is renamed in order of first use,
# and coalesce() commutes with such a renaming (aliasing, the SLOTS / TEMPS
# sets and 64-bit pair alignment are all preserved)
_COAL: Dict[str, Tuple[str, ...]] = {}
_VTOK = re.compile(r"(?<![\w.])v(?:(\d+)|\[(\d+):(\d+)\])(?![\w])")
FILE_LO, FILE_HI = G.FB, G.FB + 8 * G.NREG


def _relabel(lines: Sequence[str], blocks: Optional[Dict[int, int]] = None):
    """(lines with file blocks renamed, mapping used) — blocks: actual ->
    canonical; built in order of first appearance when None.  None when a
    register range straddles two blocks (no relabelling then)."""
    build = blocks is None
    mp: Dict[int, int] = {} if build else blocks
    bad = []

    def blk(r):
        return (r - FILE_LO) >> 3

    def sub(m):
        if m.group(1) is not None:
            r = int(m.group(1))
            if not FILE_LO <= r < FILE_HI:
                return m.group(0)
            b = blk(r)
            if b not in mp:
                if not build:
                    bad.append(r)
                    return m.group(0)
                mp[b] = len(mp)
            return "v%d" % (r + 8 * (mp[b] - b))
        lo, hi = int(m.group(2)), int(m.group(3))
        if not (FILE_LO <= lo < FILE_HI or FILE_LO <= hi < FILE_HI):
            return m.group(0)
        if not (FILE_LO <= lo and hi < FILE_HI) or blk(lo) != blk(hi):
            bad.append(lo)
            return m.group(0)
        b = blk(lo)
        if b not in mp:
            if not build:
                bad.append(lo)
                return m.group(0)
            mp[b] = len(mp)
        d = 8 * (mp[b] - b)
        return "v[%d:%d]" % (lo + d, hi + d)

    out = [_VTOK.sub(sub, l) if "v" in l else l for l in lines]
    return (None, None) if bad else (out, mp)


def coalesce_cached(hot: List[str]) -> List[str]:
    """coalesce(hot), memoised on the slot-relabelled text."""
    canon, mp = _relabel(hot)
    if canon is None:
        return coalesce(hot)
    key = "\n".join(canon)
    res = _COAL.get(key)
    if res is None:
        res = tuple(coalesce(list(canon)))
        if len(_COAL) > 100000:
            _COAL.clear()
        _COAL[key] = res
    back, _ = _relabel(res, {c: a for a, c in mp.items()})
    if back is None:                   # (cannot happen: coalesce renames within blocks)
        return coalesce(hot)
    return back


_FIELDS: Dict[int, tuple] = {}            # id(template) -> (template, fields)
_SPEC: Dict[tuple, tuple] = {}
_TAG = "@T@"


def _on_layout() -> None:
    """asmgen switched register layouts (asmgen.layout): the register-file
    and temporary ranges move, and every memo of rendered or specialised
    text belongs to the previous layout."""
    global SLOTS, TEMPS, FILE_LO, FILE_HI
    SLOTS = range(G.FB, G.FB + 8 * G.NREG)
    TEMPS = frozenset(list(range(G.XB, G.XB + 8)) + list(range(G.YB, G.TB + G.NT)))
    FILE_LO, FILE_HI = G.FB, G.FB + 8 * G.NREG
    for memo in (_TEMPLATES, _FIELDS, _SPEC, _COAL):
        memo.clear()


G._layout_hooks.append(_on_layout)


def fields_read(lines: Sequence[str]) -> Tuple[int, ...]:
    """Record words a template reads (its s40..s47 operands)."""
    key = id(lines)
    hit = _FIELDS.get(key)
    if hit is not None and hit[0] is lines:
        return hit[1]
    used = set()
    for l in lines:
        used.update(int(x) for x in re.findall(r"@F(\d)", l))
        for m in re.finditer(r"s\[?(\d+)(?::(\d+)\])?", l):
            lo = int(m.group(1))
            hi = int(m.group(2)) if m.group(2) else lo
            used.update(k - BANK0 for k in range(lo, hi + 1) if BANK0 <= k < BANK0 + 8)
        if l.startswith("@@CALL"):
            used.update((G.F_D, G.F_A, G.F_B, G.F_W, G.F_MOFF))
    _FIELDS[key] = (lines, tuple(sorted(used)))
    return _FIELDS[key][1]


def specialize_cached(name: str, var: int, rec: Sequence[int], tag: str):
    """specialize() of a record, memoised on the record words its template
    reads (records repeat across and within programs: same slots, same
    widths)."""
    lines = template(name, var)
    key = (name, var) + tuple(int(rec[k]) for k in fields_read(lines))
    hit = _SPEC.get(key)
    if hit is None:
        full = [0] * 8
        for k in fields_read(lines):
            full[k] = int(rec[k])
        hot, cold, call = specialize(lines, full, _TAG)
        hit = (coalesce_cached(hot), cold, call)
        if len(_SPEC) > 200000:
            _SPEC.clear()
        _SPEC[key] = hit
    hot, cold, call = hit
    return ([l.replace(_TAG, tag) if _TAG in l else l for l in hot],
            [l.replace(_TAG, tag) if _TAG in l else l for l in cold], call)


# ---------------------------------------------------------------------------
# programs
# ---------------------------------------------------------------------------

def decode(h: int) -> Tuple[str, int]:
    c = G.canonical(int(h))
    return G.AOPS[c // (2 * G.NVAR)], (c // 2) % G.NVAR


FP_MUL = 0x100000001B3


JIT_MAGIC = 0x4D474A4954763033             # include/mythgpu.h MG_JIT_MAGIC


def records_fingerprint(rec) -> int:
    """Fingerprint of a program's records as mg_load_program fingerprints
    them (handler ids in word 0, LEAFD records patched, zeroed pad record
    included): every word times successive powers of FP_MUL, mod 2^64, plus
    the record count.  The handler id carries the operation and its variant,
    so records that differ only in an opcode differ here.  mg_jit_attach
    refuses an image entry whose fingerprint is not the loaded program's
    (mg_api.cpp rec_fingerprint)."""
    w = np.ascontiguousarray(np.asarray(rec, dtype=np.uint64)).reshape(-1)
    with np.errstate(over="ignore"):
        pw = np.cumprod(np.full(w.size, FP_MUL, dtype=np.uint64), dtype=np.uint64)
        h = int(np.sum(w * pw, dtype=np.uint64))
    return (h + len(w) // 8) & ((1 << 64) - 1)


def program_records(prog, leafgen, prog_seed: int, lds_slots: Optional[int] = None,
                    full: bool = False):
    """The records ``mg_load_program`` uploads for ``prog`` (handler ids in
    word 0; LEAFD records patched with their leaf's generator parameters
    exactly as mg_load_program does), and the translator's mask count."""
    from .engine import lds_slots_for, translate_records
    if lds_slots is None:
        lds_slots = lds_slots_for(prog.nreg)
    rec, n_masks = translate_records(prog, I.check_lds_slots(lds_slots))
    rec = rec.reshape(-1, 8).copy()
    n_consts = prog.consts.shape[0]
    n_leaves = len(prog.leaves)
    for r in rec:
        name, var = decode(r[0])
        li = int(r[4])
        if name == "LEAFD" and li < n_leaves:
            g = leafgen[li]
            salt = ((prog_seed * 0xD1B54A32D192ED03) ^ ((li + 1) * 0x8CB92BA72F3D8DD7)) & ((1 << 64) - 1)
            r[1] = (n_consts + n_masks + 3 * g.pool_off) * 32
            r[2], r[3] = salt & M32, salt >> 32
            r[5] = g.pool_n
            r[7] = g.pct_uniform | g.pct_small << 8 | g.pct_boundary << 16
    if full:
        return rec, n_masks
    return rec[:-1], n_masks                     # the last record is the zeroed pad


CONST_SPAIR = G.BANK[1] + 4


def const_code(var: int, rec, prog) -> List[str]:
    """CONST with the value known: immediate moves instead of a scalar load
    of the constant table and its wait."""
    off = int(rec[G.F_IMM]) // 32
    limbs = [int(x) for x in prog.consts[off]] if off < prog.consts.shape[0] else None
    if limbs is None:
        raise JitUnsupported("CONST outside the program's constants")
    d = G.FB + int(rec[G.F_D])
    n = 1 if var & G.V_W32 else 8
    if var & G.V_W32 and var & G.V_DC:
        idx = [0]                               # upper limbs already zero
    else:
        idx = list(range(8))
    out = []
    vals = [limbs[j] if j < n else 0 for j in range(8)]
    for j in range(0, 8, 2):                    # pairs stay 64-bit aligned
        if j in idx and j + 1 in idx:
            # one v_mov_b64 per limb pair (4 cycles) instead of two v_mov_b32
            # (2.67 each): an inline constant when the pair is one, else the
            # pair staged in s[52:53] (record bank B: unused by compiled code
            # outside the division body, which sets it itself)
            lo, hi = vals[j], vals[j + 1]
            pair = "v[%d:%d]" % (d + j, d + j + 1)
            if hi == 0 and lo <= 64:
                out.append("    v_mov_b64 %s, %d" % (pair, lo))
            elif lo == hi == M32:
                out.append("    v_mov_b64 %s, -1" % pair)
            else:
                out.append("    s_mov_b32 s%d, 0x%x" % (CONST_SPAIR, lo))
                out.append("    s_mov_b32 s%d, 0x%x" % (CONST_SPAIR + 1, hi))
                out.append("    v_mov_b64 %s, s[%d:%d]" % (pair, CONST_SPAIR, CONST_SPAIR + 1))
            continue
        for q in (j, j + 1):
            if q in idx:
                out.append("    v_mov_b32 v%d, %s" % (d + q, _inline(vals[q]) or "0x%x" % vals[q]))
    if var & G.V_ROOT:
        out.append("    v_and_b32 %s, %s, %s" % (G.PINNED["root"], _inline(limbs[0]) or
                                                   "0x%x" % limbs[0], G.PINNED["root"]))
    return out


def program_asm(prog, leafgen, prog_seed: int, entry: str, lds_slots: Optional[int] = None,
                tag: Optional[str] = None, marks: bool = False,
                fps: Optional[List[int]] = None) -> List[str]:
    """Straight-line gfx950 code of one program, entered at label
    ``entry`` (a local ``.L`` label, or a symbol the caller declares).
    ``marks``: a label ``.Lmark_<record>_<family>_<variant>`` ahead of each
    record's code (profiling in the simulator, tools/jit_profile.py).
    ``fps``: the records' fingerprint is appended to it.  Rendered for the
    program's register layout (``Program.nreg``)."""
    with G.layout(prog.nreg):
        return _program_asm(prog, leafgen, prog_seed, entry, lds_slots, tag, marks, fps)


def _program_asm(prog, leafgen, prog_seed, entry, lds_slots, tag, marks, fps) -> List[str]:
    full, _ = program_records(prog, leafgen, prog_seed, lds_slots, full=True)
    recs = full[:-1]                             # the last record is the zeroed pad
    if fps is not None:
        fps.append(records_fingerprint(full))
    tag = tag or entry.lstrip(".L")
    out = [entry + ":"]
    # s[S_FAST] bit 0: generator mode, no leaf store and a wave whose
    # first active index starts a group of 64 (every active lane in one
    # group) — the one test a compiled LEAFD makes on its common path
    # (asmgen.h_leafd); s[S_GROUP] = lo32(that index >> 6), the group
    # the leaves' classes are drawn for
    g = G.S_GROUP
    out.append("    s_cmp_eq_u64 %s, 0" % G.PINNED["lout"])
    out.append("    s_cselect_b32 s%d, %s, 0" % (G.S_FAST, G.PINNED["mode"]))
    out.append("    v_readfirstlane_b32 s%d, %s" % (g, G.PINNED["idx_lo"]))
    out.append("    v_readfirstlane_b32 s%d, %s" % (g + 1, G.PINNED["idx_hi"]))
    out.append("    s_and_b32 s%d, s%d, 63" % (G.S_T, g))
    out.append("    s_cselect_b32 s%d, 0, s%d" % (G.S_FAST, G.S_FAST))
    out.append("    s_lshr_b64 s[%d:%d], s[%d:%d], 6" % (g, g + 1, g, g + 1))
    pending_cold: List[str] = []
    flush_no = 0
    for i, r in enumerate(recs):
        name, var = decode(r[0])
        if marks:
            out.append(".Lmark_%d_%s_%d:" % (i, name, var))
        if name == "CONST":
            hot, cold = const_code(var, r, prog), []
        else:
            hot, cold, _ = specialize_cached(name, var, r, "%s_%d" % (tag, i))
        out.extend(hot)
        pending_cold.extend(cold)
        if name == "HALT" or (pending_cold and (i + 1) % COLD_FLUSH == 0):
            if name != "HALT":
                skip = ".L%s_k%d" % (tag, flush_no)
                out.append("    s_branch %s" % skip)
                out.extend(pending_cold)
                out.append(skip + ":")
            else:
                out.extend(pending_cold)
            pending_cold = []
            flush_no += 1
        if name == "HALT":
            break
    return peephole(out)


_WIDE_STORE = re.compile(r"(scratch|global|flat|buffer)_store_dwordx[34]\b")


def peephole(lines: List[str]) -> List[str]:
    """Drop ``s_waitcnt lgkmcnt(0)`` where no LDS / scalar-memory operation
    was issued since the last one on the straight path (a label or a call
    counts as possibly pending), and keep one wait state between a vector-
    memory store of more than 64 bits and a following VALU instruction (the
    store reads its data VGPRs after issue: a VALU write to them in the next
    cycle would corrupt the stored data — the interpreter's dispatch gave
    that slack for free; straight-line code must ask for it)."""
    out, pending = [], True
    for n, l in enumerate(lines):
        t = l.strip()
        if out and _WIDE_STORE.match(out[-1].strip()) and t.startswith("v_"):
            out.append("    s_nop 0")
        if t.endswith(":") or t.startswith(("s_load", "ds_", "s_swappc")):
            pending = True
        elif t == "s_waitcnt lgkmcnt(0)":
            if not pending:
                continue
            pending = False
        out.append(l)
    return out


HEADER = '\t.amdgcn_target "amdgcn-amd-amdhsa--%s"\n' % ARCH


def chunk_asm(items, first: int, lds_slots: Optional[int] = None,
              fps: Optional[List[int]] = None) -> str:
    """One object's worth of programs: program ``first + i`` is entered at
    the (hidden) symbol ``mg_jp<first+i>``; the shared heavy bodies are
    copied into every chunk (local labels, a few KiB).  The programs' record
    fingerprints are appended to ``fps``.  The programs share one register
    layout (the bodies are rendered for it)."""
    nreg = _batch_layout(p for p, _, _ in items)
    with G.layout(nreg):
        return _chunk_asm(items, first, lds_slots, fps)


def _batch_layout(progs) -> int:
    """The one register layout of a batch's programs (a batch runs on one
    context, Engine(nreg))."""
    ns = {p.nreg for p in progs}
    if len(ns) > 1:
        raise ValueError("a batch mixes register layouts %s" % sorted(ns))
    return ns.pop() if ns else G.NREG


def _chunk_asm(items, first: int, lds_slots: int, fps: Optional[List[int]]) -> str:
    parts = [HEADER, "\t.text\n\t.p2align 8\n"]
    for i, (p, g, s) in enumerate(items):
        sym = "mg_jp%d" % (first + i)
        fp: List[int] = []
        try:
            text = program_asm(p, g, s, sym, lds_slots, tag="p%d" % (first + i), fps=fp)
        except JitUnsupported:
            fp = [None]               # stays on the interpreter: a zero table row
            text = None
        if fps is not None:
            fps.append(fp[0])
        if text is None:
            continue
        parts.append("\t.globl %s\n\t.hidden %s\n" % (sym, sym))
        parts.append("\n".join(text))
        parts.append("\n")
    parts.append("\t.p2align 6\n" + "\n".join(bodies()) + "\n")
    return "".join(parts)


def table_asm(fps: Sequence[Optional[int]], nreg: Optional[int] = None) -> str:
    """The stub kernel and ``mg_jit_table``: a header row (JIT_MAGIC, the
    interpreter's asm digest: the code is generated from its handlers and
    assumes its pinned registers and descriptor layout), then row i + 1 =
    (mg_jp<i> - table, fingerprint of program i's records), or (0, 0) for a
    program that was not compiled (JitUnsupported: mg_jit_attach leaves it on
    the interpreter).  ``nreg``: the programs' register layout."""
    stub = open(STUB).read()
    cut = stub.index("\t.ident")
    with G.layout(G.NREG if nreg is None else nreg):
        dg = G.digest()
    head = "\t.quad 0x%x\n\t.quad 0x%s\n" % (JIT_MAGIC, dg[:16])
    rows = "".join(("\t.quad mg_jp%d - . + %d\n\t.quad 0x%x\n" % (i, 16 * (i + 1), fp))
                   if fp is not None else "\t.quad 0\n\t.quad 0\n" for i, fp in enumerate(fps))
    return (stub[:cut] + "\t.data\n\t.globl mg_jit_table\n\t.protected mg_jit_table\n"
            "\t.type mg_jit_table,@object\n\t.p2align 3\nmg_jit_table:\n" + head + rows +
            "\t.size mg_jit_table, %d\n" % (16 * (len(fps) + 1)) + stub[cut:])


def _as(text: str, obj: str) -> None:
    src = obj[:-2] + ".s"
    with open(src, "w") as fh:
        fh.write(text)
    subprocess.run([os.path.join(LLVM_BIN, "clang"), "-cc1as", "-triple", "amdgcn-amd-amdhsa",
                    "-target-cpu", ARCH, "-filetype", "obj", src, "-o", obj], check=True)


def _chunk_job(args):
    items, first, lds_slots, obj = args
    if any(g is None for _, g, _ in items):
        from .engine import default_leafgen
        items = [(p, default_leafgen(p) if g is None else g, s) for p, g, s in items]
    fps: List[int] = []
    _as(chunk_asm(items, first, lds_slots, fps), obj)
    return obj, fps


def source_digest() -> str:
    """Digest of everything a compiled image depends on: the Python compiler
    and generator sources, the C++ translator (the records), the public
    headers (IR and descriptor layout), the generated interpreter's own
    digest, and the environment knobs that change rendered handler bodies or
    programs (a cached image must not survive an A/B knob)."""
    import hashlib
    h = hashlib.sha1(ARCH.encode())
    pkg = os.path.dirname(os.path.abspath(__file__))
    inc = os.path.join(os.path.dirname(pkg), "include")
    for d in (pkg, os.path.join(pkg, "smt"), os.path.join(pkg, "csrc"), inc):
        for f in sorted(os.listdir(d)):
            if f.endswith((".py", ".cpp", ".h")):
                with open(os.path.join(d, f), "rb") as fh:
                    h.update(f.encode() + fh.read())
    from . import ir
    asm = {}
    for n in (16, 11):
        with G.layout(n):
            asm[n] = G.digest()
    knobs = {"flush": COLD_FLUSH, "asm": sorted(asm.items()), "leaf_remat": ir.LEAF_REMAT}
    h.update(repr(sorted(knobs.items())).encode())
    return h.hexdigest()[:16]


CODE_FILES = ("jit.py", "asmgen.py", "irdefs.py", "engine.py", "csrc/mg_host.cpp",
              "csrc/mg_api.cpp")


def code_digest() -> str:
    """Digest of the sources that turn an IR program into compiled code
    (handler generator, specialiser, leaf-generator parameters, record
    translator); the programs themselves are keyed by content
    (bench.programs_digest).  bench.py keys traffic measurements on both
    (profiles/traffic.json)."""
    import hashlib
    h = hashlib.sha1(ARCH.encode())
    pkg = os.path.dirname(os.path.abspath(__file__))
    for f in CODE_FILES:
        with open(os.path.join(pkg, f), "rb") as fh:
            h.update(f.encode() + fh.read())
    return h.hexdigest()[:16]


def cached_image(key: str, build, cache_dir: Optional[str] = None) -> Tuple[bytes, bool]:
    """(image, was_cached): ``build()``'s code object, memoised in
    ``<dir>/<key>_<source digest>.hsaco`` when a directory is given
    (``cache_dir``, else ``$MYTHGPU_JIT_CACHE``).  Profiling runs assemble the
    image in a separate step, so a process the profiler has already attached
    to the GPU never starts the assembler; the ranks of one node share one
    build: the file is made under an exclusive ``flock`` of ``<path>.lock``,
    so the first rank builds while the others wait and then read it.
    ``key`` must identify the programs (workload, ids); the source digest is
    added here."""
    d = cache_dir or os.environ.get("MYTHGPU_JIT_CACHE")
    if not d:
        return build(), False
    import fcntl
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, "%s_%s.hsaco" % (re.sub(r"[^\w.-]", "_", key), source_digest()))
    with open(path + ".lock", "a+") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            if os.path.exists(path):
                with open(path, "rb") as fh:
                    return fh.read(), True
            image = build()
            tmp = path + ".tmp%d" % os.getpid()
            with open(tmp, "wb") as fh:
                fh.write(image)
            os.replace(tmp, path)
            return image, False
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


def compile_batch(items, lds_slots: Optional[int] = None, workers: int = 1, chunk: int = 64,
                  start: str = "fork") -> bytes:
    """gfx950 code object of [(program, leafgen or None (= the C2 default),
    prog_seed)], entries in order (``Engine.jit_attach`` takes the same
    programs in the same order).  Chunks of programs are rendered and
    assembled on ``workers`` host processes (``start="fork"`` before the
    process touches the GPU, ``"spawn"`` after), then linked with the table
    into one shared object.  ``lds_slots``: the LDS spill regions of the
    context the programs will run on (default: their layout's,
    engine.lds_slots_for)."""
    if lds_slots is None:
        from .engine import lds_slots_for
        lds_slots = lds_slots_for(_batch_layout(p for p, _, _ in items))
    if workers > 1:                   # enough chunks to keep every worker busy
        chunk = max(1, min(chunk, -(-len(items) // (4 * workers))))
    with tempfile.TemporaryDirectory() as d:
        jobs = [(list(items[i:i + chunk]), i, lds_slots, os.path.join(d, "c%d.o" % i))
                for i in range(0, len(items), chunk)]
        from .procmap import process_map
        objs = process_map(_chunk_job, jobs, workers, start)
        fps = [fp for _, f in objs for fp in f]
        objs = [o for o, _ in objs]
        tab = os.path.join(d, "table.o")
        _as(table_asm(fps, _batch_layout(p for p, _, _ in items)), tab)
        out = os.path.join(d, "jit.hsaco")
        subprocess.run([os.path.join(LLVM_BIN, "ld.lld"), "-shared", tab] + objs + ["-o", out],
                       check=True)
        with open(out, "rb") as fh:
            return fh.read()
