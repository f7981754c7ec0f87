"""Generator of the hand-written gfx950 (CDNA4) assembly interpreter for the
mythgpu IR — the engine's hot kernel.

Why assembly: on MI355X every instruction a wave issues, scalar or vector,
costs ~4 SIMD cycles (``profiles/r01/ubench.log``).  The compiled C++
interpreter spent ~40 scalar instructions per IR op on decoding and a binary
search dispatch plus ~30 vector moves on register-file copies.  This one is
written instruction by instruction:

* **direct-threaded dispatch**: the host translates each IR instruction into
  an 8-word record whose first word is the byte offset of its handler; every
  handler ends with ``s_add_u32 / s_addc_u32 / s_setpc_b64`` to the next.
  The next record is prefetched (``s_load_dwordx8``) into the other of two
  SGPR banks at handler entry, so each handler exists in a bank-A and a
  bank-B variant (heavy ops copy their record and always prefetch into A);
* **pre-decoded fields**: register slots arrive as GPR-index values
  (8 x slot); uniform shifts, funnel indices and constant-pool offsets are
  computed by the translator (``mg_api.cpp``);
* **GPR-indexed ALU**: one operand is consumed straight from the register
  file by the arithmetic (``s_set_gpr_idx_on ... gpr_idx(SRC0)``), only the
  other is copied; EXTRACT/CONCAT are one ``v_alignbit_b32`` per limb with
  both sources indexed;
* **variants**: ROOT-fused and width-masked forms of every handler, chosen
  by the translator, so the common 256-bit non-root case pays nothing.

Register file: 16 slots x 8 limbs at v[8 + 8*slot + limb]; X (v0..v7) and
Y (v136..v143) double as guards below/above it for the funnel reads.

This module writes ``csrc/mg_interp_gfx950.inc`` (the assembly, as the body
of the inline asm in ``mg_interp_asm.hip``) and ``csrc/mg_asm_handlers.h``
(handler numbering shared with the translator).  It runs at build time only
(``mythril_amd/build.py``).
"""

from __future__ import annotations

import os
import re
from typing import Dict, List, Optional

# register-file slots of the layout being generated (MG_NREG = 16, or 11:
# the four-wave layout; ``layout()`` switches, the library holds both);
# MYTHGPU_NREG sets the process's default layout
NREG = int(os.environ.get("MYTHGPU_NREG", "16"))
FB = 8                     # first VGPR of the file
XB = 0                     # X temps v0..v7   (guard below the file)
YB = FB + 8 * NREG         # Y temps v136..v143 (guard above the file)
RB = YB + 8                # R temps v144..v151
TB = RB + 8                # T temps v152..v163
NT = 12
NVGPR_FIXED = TB + NT      # v0..v163 named here; root/lane/lds are operands

# ---- SGPR plan (inputs are inline-asm operands used in place) --------------
BANK = (40, 48)            # s[40:47], s[48:55]: the two record banks
S_BASE = 56                # s[56:57] handler base PC
S_CODE = 58                # s[58:59] translated code
S_IP = 60                  # byte offset of the next record to prefetch
S_FAST = S_IP              # compiled programs (no prefetch): bit 0 = generator
                           # mode, no leaf store, wave group aligned to 64
                           # candidates (jit.program_asm sets it)
S_VAR = 61                 # heavy ops: variant bits | op << 4
S_CONST = 62               # s[62:63] constant pool
S_CUR = 64                 # s[64:71] current record of a heavy op / LEAF descriptor
S_M = 72                   # s[72:79] width masks (8)
S_T = 80                   # s[80:87] temps; s[86:87] is also the jump target
S_X = 88                   # s[88:95] division lane masks (ns, nt, z) + op
S_JMP = S_T + 6
S_M0 = S_X + 7             # m0 (GPR-index register) saved across the asm
S_K = 96                   # s[96:101] SplitMix64 constants, set once at entry
S_LAST = S_K + 5

F_OFF, F_D, F_A, F_B, F_C, F_IMM, F_W, F_MOFF = range(8)
# LEAFD records carry the leaf's generator parameters (mg_load_program
# patches them in): pool offset, salt pair, pool size, thresholds
# (uniform | small << 8 | boundary << 16); C is the leaf index, W the wait flag
LEAFD_POFF, LEAFD_SALT, LEAFD_PN, LEAFD_PCT = 1, 2, 5, 7

AOPS = ["NOP", "HALT", "CONST", "LEAF", "SPILL_LDS", "SPILL_SCR", "RELOAD_LDS", "RELOAD_SCR",
        "ADD", "SUB", "MUL", "UDIV", "UREM", "SDIV", "SREM", "SMOD", "AND", "OR", "XOR",
        "NOT", "SHL", "LSHR", "ASHR", "EQ", "ULT", "ULE", "SLT", "SLE", "UMULNO", "ITE",
        "CONCAT", "EXTRACT", "SEXT", "NEG", "OUT", "ROOT", "MOV",
        "SUBR",     # b - a   (SUB with the operands swapped: in place on a)
        "ITEN",     # c ? b : a (ITE with the operands swapped: in place on a)
        "LEAFD",    # 256-bit LEAF straight into slot = variant, loads left in flight
        "WAITVM",   # wait for in-flight LEAFD / RELOADD loads (inserted by the translator)
        "RELOADD",  # scratch reload straight into slot = variant, loads left in flight
        "EQSEL",    # fused EQ + ITE of a store-chain link (translator): see h_eqsel
        "EXTRACTN",  # EXTRACT to W > 32 bits: variant = result limbs - 1
        "CONCATQ",  # CONCAT: variant = limb shift q | 8 if a bit shift remains
        "BCAST",    # the calldata word (mythgpu_ir.h MG_BCAST / MG_CDWE / MG_CDWX)
        "CDWE",
        "CDWX"]
AOP = {n: i for i, n in enumerate(AOPS)}
V_ROOT, V_MASK, V_DC, V_W32, V_IP = 1, 2, 4, 8, 16
# NW = a ROOT-fused result nobody reads: only the root is updated, the slot
# is not written (chosen by the translator, mg_host.cpp)
V_NW = 32
NVAR = 64
# variant bits each handler family implements (the query maps the others to
# the nearest implemented handler): DC = destination's upper limbs are known
# zero (write limb 0 only), W32 = operands and result fit one limb
_RM = V_ROOT | V_MASK
SUPPORT = {n: _RM for n in AOPS}
SUPPORT.update({n: _RM | V_DC | V_W32 for n in ("ADD", "SUB", "AND", "OR", "XOR", "NOT", "NEG",
                                               "ITE", "EQ", "ULT", "ULE", "EXTRACT", "MOV",
                                               "CONST")})
SUPPORT.update({n: _RM | V_DC for n in ("SLT", "SLE")})
# IP = the destination is operand a's slot: the ALU op writes the file in place
SUPPORT.update({n: SUPPORT[n] | V_IP for n in ("ADD", "SUB", "AND", "OR", "XOR", "NOT", "NEG",
                                               "ITE")})
for _n in ("EQ", "ULT", "ULE", "SLT", "SLE", "AND", "OR", "XOR"):
    SUPPORT[_n] |= V_NW
SUPPORT["SUBR"] = _RM | V_IP
SUPPORT["BCAST"] = 0
SUPPORT["CDWE"] = SUPPORT["CDWX"] = V_IP        # 256-bit results, never ROOT
SUPPORT["ITEN"] = V_ROOT | V_IP
SUPPORT["WAITVM"] = 0
V_NEG, V_GEN = 1, 2          # EQSEL: copy where not equal / three-address form
SUPPORT["EQSEL"] = V_NEG | V_GEN
# families whose result is never masked (canonical inputs give canonical
# outputs) and families where DC only matters for one-limb results
NO_MASK = {"AND", "OR", "XOR", "EQ", "ULT", "ULE", "ITE", "ITEN", "MOV", "CONST", "NOP", "HALT",
           "SPILL_LDS", "SPILL_SCR", "RELOAD_LDS", "RELOAD_SCR", "OUT", "ROOT", "CONCAT",
           "EXTRACT"}
DC_NEEDS_W32 = {"ADD", "SUB", "AND", "OR", "XOR", "NOT", "NEG", "ITE", "EXTRACT", "MOV", "CONST"}


# families whose variant is a register slot (static registers in the handler)
SLOT_VARIANT = {"LEAFD", "RELOADD", "SPILL_LDS", "SPILL_SCR", "RELOAD_LDS"}


# LEAFD / RELOADD: variant = slot | WAITD when the handler waits for its own
# loads (its consumer is the very next record; the translator folds the wait)
V_WAITD = 16
# SPILL_SCR / RELOADD: the value is one limb (limbs 1..7 zero): one dword of
# scratch instead of eight (the translator decides at the spill)
V_NARROW = 32


def canon_var(name: str, var: int) -> int:
    if name == "LEAFD":
        return var & (V_WAITD | 15) if (var & 15) < NREG else 0
    if name == "RELOADD":
        return var & (V_NARROW | V_WAITD | 15) if (var & 15) < NREG else 0
    if name in ("SPILL_SCR", "SPILL_LDS", "RELOAD_LDS"):
        return var & (V_NARROW | 15) if (var & 15) < NREG else 0
    if name in SLOT_VARIANT:
        return var if var < NREG else 0      # the variant is the register slot
    if name == "EXTRACTN":
        return var & 7
    if name == "CONCATQ":
        return var & 15
    var &= SUPPORT[name]
    if name in NO_MASK:
        var &= ~V_MASK
    if name in DC_NEEDS_W32 and not var & V_W32:
        var &= ~V_DC
    if var & V_W32:
        var &= ~V_IP                 # one limb: nothing to save
    if not var & V_ROOT:
        var &= ~V_NW                 # only a ROOT-fused result can go unwritten
    if var & V_NW:
        var &= ~V_DC
        if name in ("AND", "OR", "XOR") and not var & V_W32:
            var &= ~V_NW             # Bool logic is one limb
    return var


def hid(aop: int, variant: int, bank: int) -> int:
    return (aop * NVAR + variant) * 2 + bank


NUM_HANDLERS = len(AOPS) * NVAR * 2


def canonical(h: int) -> int:
    """The implemented handler a handler id maps to (unsupported variant
    bits dropped)."""
    bank, var, aop = h % 2, (h // 2) % NVAR, h // (2 * NVAR)
    return hid(aop, canon_var(AOPS[aop], var), bank)


def v(n: int) -> str:
    return "v%d" % n


def s(n: int) -> str:
    return "s%d" % n


def sp(n: int) -> str:
    return "s[%d:%d]" % (n, n + 1)


def vp(n: int) -> str:
    return "v[%d:%d]" % (n, n + 1)


X = [XB + j for j in range(8)]
Y = [YB + j for j in range(8)]
R = [RB + j for j in range(8)]
T = [TB + j for j in range(NT)]
F = [FB + j for j in range(8)]          # limb j of the indexed slot (index = 8*slot)
G = [FB - 8 + j for j in range(10)]     # funnel base (index = 8*slot + limb shift + 8)
TMP = T[11]

# inline-asm operand names
# idx = the lane's candidate index (first + lane, 64-bit; the C++ shell)
OP_ROOT, OP_IDX_LO, OP_IDX_HI, OP_LDS = "%[root]", "%[idx_lo]", "%[idx_hi]", "%[lds]"
IN = {k: "%%[%s]" % k for k in ("desc", "seed", "first", "leaves", "stride", "lout", "probes",
                                "mode", "scr", "active", "table")}
# Every operand lives in a FIXED register (physical-register constraints in
# mg_interp_asm.hip, generated from this table): compiled programs (jit.py),
# assembled apart from the kernel, address them by these names too.
PINNED = {"root": v(NVGPR_FIXED), "idx_lo": v(NVGPR_FIXED + 1), "idx_hi": v(NVGPR_FIXED + 2),
          "lds": v(NVGPR_FIXED + 3),
          "desc": "s[16:17]", "seed": "s[18:19]", "first": "s[20:21]", "leaves": "s[22:23]",
          "stride": "s[24:25]", "lout": "s[26:27]", "probes": "s[28:29]", "mode": "s30",
          "scr": "s31", "active": "s[32:33]", "table": "s[34:35]"}
NVGPR_KERNEL = NVGPR_FIXED + 4   # the kernel's VGPR budget (168: 3 waves / SIMD)


# Layout switching: every name below derives from NREG; functions read them
# as module globals at call time, so rebinding them switches what generate(),
# digest(), canonical() and the compiled-program renderer (jit.py, which
# registers a hook for its own derived tables and caches) produce.
_layout_hooks = []


def _set_layout(nreg: int) -> None:
    global NREG, YB, RB, TB, NVGPR_FIXED, Y, R, T, TMP, PINNED, NVGPR_KERNEL
    NREG = nreg
    YB = FB + 8 * NREG
    RB = YB + 8
    TB = RB + 8
    NVGPR_FIXED = TB + NT
    Y = [YB + j for j in range(8)]
    R = [RB + j for j in range(8)]
    T = [TB + j for j in range(NT)]
    TMP = T[11]
    PINNED = dict(PINNED, root=v(NVGPR_FIXED), idx_lo=v(NVGPR_FIXED + 1),
                  idx_hi=v(NVGPR_FIXED + 2), lds=v(NVGPR_FIXED + 3))
    NVGPR_KERNEL = NVGPR_FIXED + 4
    for hook in _layout_hooks:
        hook()


class layout:
    """``with asmgen.layout(11): ...`` generates for the 11-slot layout and
    restores the previous one on exit (not thread-safe: renderers switch it
    in one thread, worker processes have their own)."""

    def __init__(self, nreg: int):
        if nreg not in (16, 11):
            raise ValueError("no %d-slot register layout (16, 11)" % nreg)
        self.nreg = nreg

    def __enter__(self):
        self.prev = NREG
        if self.nreg != NREG:
            _set_layout(self.nreg)
        return self

    def __exit__(self, *exc):
        if NREG != self.prev:
            _set_layout(self.prev)
        return False
# mg_pdesc byte offsets the assembly reads (mg_device.h)
PDESC_CONSTS, PDESC_XCODE, PDESC_BTAB, PDESC_JIT = 0x8, 0x30, 0x38, 0x40

# Compiled-program (JIT) generation mode, set by mythril_amd/jit.py while it
# renders handler templates: no record prefetch, no dispatch (a marker line
# ends the handler's straight-line part), heavy stubs become call markers.
JIT = False
JIT_RET = 58               # s[58:59]: return address into the interpreter
JIT_BODY_RET = 56          # s[56:57]: return address of a shared heavy body


class Asm:
    def __init__(self):
        self.lines: List[str] = []
        self._n = 0
        self._hot: Optional[List[str]] = None
        self._cold: List[str] = []
        self._idx_state = None
        self.nw = False              # the handler being generated is an NW variant
        # GPR-index mode may still be on at a handler's entry (a handler
        # leaves it on when its last VGPR access was indexed: dispatch drops
        # the trailing s_set_gpr_idx_off); the first instruction that touches
        # VGPRs before the handler sets the mode itself gets the off first
        self._entry_idx_unknown = False

    def __call__(self, text: str):
        if self._entry_idx_unknown:
            op = text.split(None, 1)[0]
            if op.startswith("s_set_gpr_idx_on") or op == "s_set_gpr_idx_off":
                self._entry_idx_unknown = False
            elif (not op.startswith("s_") and not op.startswith(".")) or \
                    op.startswith("s_cbranch") or op == "s_branch":
                # before the first VGPR access, or before a branch (a path
                # that leaves the straight line must not miss it)
                self._entry_idx_unknown = False
                self.lines.append("    s_set_gpr_idx_off")
        self.lines.append("    " + text)

    def label(self, name: str):
        if name.startswith(".Lh") or name.startswith(".Lbody_"):
            self._entry_idx_unknown = True       # entered from any handler's dispatch
        self.lines.append(name + ":")

    def cold(self):
        """Following lines go out of line (a rarely taken block), until
        :meth:`hot`; :meth:`flush_cold` places them after the body's final
        dispatch, so the common path runs straight through."""
        self._hot, self.lines = self.lines, self._cold

    def hot(self):
        self.lines, self._hot = self._hot, None

    def flush_cold(self):
        self.lines.extend(self._cold)
        self._cold = []

    def uniq(self, stem: str) -> str:
        self._n += 1
        return ".L%s%d_%%=" % (stem, self._n)

    def idx_on(self, sreg: int, mode: str):
        """GPR-index mode on.  Right after an idx_off whose on-state is
        known, the pair becomes one instruction: s_set_gpr_idx_idx (same
        mode, another index) or s_set_gpr_idx_mode (same index)."""
        after_off = bool(self.lines) and self.lines[-1].strip() == "s_set_gpr_idx_off"
        prev = self._idx_state if after_off else None
        self._idx_state = None
        if after_off:
            # s_set_gpr_idx_on sets index and mode whatever the state: an off
            # right before it is redundant
            self.lines.pop()
        if prev is not None and (prev[1] == mode or prev[0] == sreg):
            if prev[1] != mode:
                self("s_set_gpr_idx_mode gpr_idx(%s)" % mode)
            elif prev[0] != sreg:
                self("s_set_gpr_idx_idx %s" % s(sreg))
            return
        self("s_set_gpr_idx_on %s, gpr_idx(%s)" % (s(sreg), mode))

    def idx_off(self):
        # the on-state being closed, if no label or other index change
        # came after the s_set_gpr_idx_on (a following idx_on may merge)
        st = None
        for line in reversed(self.lines):
            t = line.strip()
            m = re.fullmatch(r"s_set_gpr_idx_on s(\d+), gpr_idx\(([A-Z0-9,]+)\)", t)
            if m:
                st = (int(m.group(1)), m.group(2))
                break
            if t.startswith("s_set_gpr_idx_") or t.endswith(":"):
                break
        self("s_set_gpr_idx_off")
        self._idx_state = st

    def read_slot(self, dst: List[int], fld_sgpr: int):
        """dst[0..7] <- F[slot] with four 64-bit moves (full rate on gfx950,
        profiles/r01/ubench2.log; slot indices keep pairs aligned)."""
        self.idx_on(fld_sgpr, "SRC0")
        for j in range(0, 8, 2):
            self("v_mov_b64 %s, %s" % (vp(dst[j]), vp(F[j])))
        self.idx_off()

    def write_slot(self, src: List[int], fld_sgpr: int, masks: Optional[int] = None):
        self.idx_on(fld_sgpr, "DST")
        for j in range(0, 8, 2) if masks is None else range(8):
            if masks is None:
                self("v_mov_b64 %s, %s" % (vp(F[j]), vp(src[j])))
            else:
                self("v_and_b32 %s, %s, %s" % (v(F[j]), s(masks + j), v(src[j])))
        self.idx_off()

    def root_and(self, reg: str):
        self("v_and_b32 %s, %s, %s" % (OP_ROOT, reg, OP_ROOT))


def fld(bank: int, k: int) -> int:
    return BANK[bank] + k


def cur(k: int) -> int:
    return S_CUR + k


# ---------------------------------------------------------------------------
# scaffolding
# ---------------------------------------------------------------------------

def prologue(a: Asm, bank: int):
    if JIT:
        return
    ob = BANK[1 - bank]
    a("s_load_dwordx8 s[%d:%d], %s, %s" % (ob, ob + 7, sp(S_CODE), s(S_IP)))
    a("s_add_u32 %s, %s, 32" % (s(S_IP), s(S_IP)))


def dispatch(a: Asm, next_bank: int):
    if JIT:
        # end of the handler's straight-line part: the dispatch's wait stays
        # (handlers leave LDS reloads to it; jit.peephole drops the
        # redundant ones) and the mode is left off
        if not (a.lines and a.lines[-1].strip() == "s_set_gpr_idx_off"):
            a("s_set_gpr_idx_off")
        a("s_waitcnt lgkmcnt(0)")
        a.lines.append("@@END")
        return
    nb = BANK[next_bank]
    if a.lines and a.lines[-1].strip() == "s_set_gpr_idx_off":
        a.lines.pop()                  # the next handler turns it off if it must
    a("s_waitcnt lgkmcnt(0)")
    a("s_add_u32 %s, %s, %s" % (s(S_JMP), s(S_BASE), s(nb + F_OFF)))
    a("s_addc_u32 %s, %s, 0" % (s(S_JMP + 1), s(S_BASE + 1)))
    a("s_setpc_b64 %s" % sp(S_JMP))


def load_masks(a: Asm, moff_sgpr: int, dst: int = S_M):
    a("s_load_dwordx8 s[%d:%d], %s, %s" % (dst, dst + 7, sp(S_CONST), s(moff_sgpr)))


def finish(a: Asm, bank: int, res: List[int], root: bool, mask: bool):
    if mask:
        a("s_waitcnt lgkmcnt(0)")
    a.write_slot(res, fld(bank, F_D), S_M if mask else None)
    if root:
        a.root_and(v(res[0]))
    dispatch(a, 1 - bank)


def write_narrow(a: Asm, bank: int, r0: str, dc: bool):
    """F[D] = (r0, 0, ..., 0); with dc the upper limbs are already zero.
    The first pair is one v_pk_mov_b32 of r0's half and an inline zero."""
    if dc:
        a.idx_on(fld(bank, F_D), "DST")
        a("v_mov_b32 %s, %s" % (v(F[0]), r0))
        a.idx_off()
        return
    m = re.fullmatch(r"v(\d+)", r0)
    if not m:
        a("v_mov_b32 %s, %s" % (v(R[0]), r0))
        r0 = v(R[0])
    n = int(re.fullmatch(r"v(\d+)", r0).group(1))
    a.idx_on(fld(bank, F_D), "DST")
    a("v_pk_mov_b32 %s, %s, 0 op_sel:[%d,0]" % (vp(F[0]), vp(n & ~1), n & 1))   # (r0, 0)
    for j in range(2, 8, 2):
        a("v_mov_b64 %s, 0" % vp(F[j]))
    a.idx_off()


def finish_narrow(a: Asm, bank: int, root: bool, mask: bool, dc: bool):
    """R0 (one limb) -> F[D], masked to W bits if requested, ROOT, dispatch.
    NW (a dead ROOT-fused Bool): the root only."""
    if a.nw:
        a.root_and(v(R[0]))
        dispatch(a, 1 - bank)
        return
    if mask:
        a("s_waitcnt lgkmcnt(0)")
        a("v_and_b32 %s, %s, %s" % (v(R[0]), s(S_M), v(R[0])))
    write_narrow(a, bank, v(R[0]), dc)
    if root:
        a.root_and(v(R[0]))
    dispatch(a, 1 - bank)


def narrow_binop(a: Asm, bank: int, root: bool, mask: bool, dc: bool, opname: str):
    """R0 = op(F[a].limb0, F[b].limb0) for values of at most 32 bits."""
    prologue(a, bank)
    if mask:
        load_masks(a, fld(bank, F_MOFF))
    a.idx_on(fld(bank, F_B), "SRC0")
    a("v_mov_b32 %s, %s" % (v(Y[0]), v(F[0])))
    a("s_set_gpr_idx_idx %s" % s(fld(bank, F_A)))
    a("%s %s, %s, %s" % (opname, v(R[0]), v(F[0]), v(Y[0])))
    a.idx_off()
    finish_narrow(a, bank, root, mask, dc)


def sext(a: Asm, regs: List[int], wsgpr: int, masks: int, tmp: int, st: int):
    """Sign-extend regs (canonical at the width in s[wsgpr]) to 256 bits in
    place.  masks: 8 SGPRs with the bits < width; st: 2 scratch SGPRs.
    Preserves vcc."""
    a("s_sub_u32 %s, %s, 1" % (s(st), s(wsgpr)))
    a("s_lshr_b32 %s, %s, 5" % (s(st + 1), s(st)))
    a("s_and_b32 %s, %s, 31" % (s(st), s(st)))
    a("s_set_gpr_idx_on %s, gpr_idx(SRC0)" % s(st + 1))
    a("v_mov_b32 %s, %s" % (v(tmp), v(regs[0])))
    a.idx_off()
    a("v_bfe_u32 %s, %s, %s, 1" % (v(tmp), v(tmp), s(st)))
    a("v_sub_u32 %s, 0, %s" % (v(tmp), v(tmp)))
    for j in range(8):
        a("v_bfi_b32 %s, %s, %s, %s" % (v(regs[j]), s(masks + j), v(regs[j]), v(tmp)))


def or_reduce(a: Asm, regs: List[int], out: int):
    a("v_or3_b32 %s, %s, %s, %s" % (v(out), v(regs[0]), v(regs[1]), v(regs[2])))
    a("v_or3_b32 %s, %s, %s, %s" % (v(out), v(out), v(regs[3]), v(regs[4])))
    a("v_or3_b32 %s, %s, %s, %s" % (v(out), v(out), v(regs[5]), v(regs[6])))
    a("v_or_b32 %s, %s, %s" % (v(out), v(out), v(regs[7])))


# ---------------------------------------------------------------------------
# cheap handlers (a, bank, root, mask)
# ---------------------------------------------------------------------------

def h_nop(a, bank, root, mask, dc=False, w32=False, ip=False):
    prologue(a, bank)
    dispatch(a, 1 - bank)


def h_halt(a, bank, root, mask, dc=False, w32=False, ip=False):
    a("s_waitcnt lgkmcnt(0)")
    if JIT:
        a.lines.append("@@HALT")
        return
    far_jump(a, ".Lexit_%=")           # the handlers outgrow s_branch's range


def h_const(a, bank, root, mask, dc=False, w32=False, ip=False):
    prologue(a, bank)
    load_masks(a, fld(bank, F_IMM))                # the constant itself
    a("s_waitcnt lgkmcnt(0)")
    if w32:
        write_narrow(a, bank, s(S_M), dc)
        if root:
            a.root_and(s(S_M))
        dispatch(a, 1 - bank)
        return
    a.idx_on(fld(bank, F_D), "DST")
    for j in range(0, 8, 2):
        a("v_mov_b64 %s, %s" % (vp(F[j]), sp(S_M + j)))
    a.idx_off()
    if root:
        a.root_and(s(S_M))
    dispatch(a, 1 - bank)


def _binop(a, bank, root, mask, emit):
    prologue(a, bank)
    if mask:
        load_masks(a, fld(bank, F_MOFF))
    a.read_slot(Y, fld(bank, F_B))
    a.idx_on(fld(bank, F_A), "SRC0")
    emit()
    a.idx_off()
    finish(a, bank, R, root, mask)


def inplace_op(a: Asm, bank: int, root: bool, mask: bool, mode: str, emit):
    """F[a] = op(F[a], Y) in place (dest == a): Y <- F[b]; one pass with
    the file both read and written through GPR indexing (mode: which
    source position reads F[a]); mask and ROOT applied afterwards."""
    prologue(a, bank)
    if mask:
        load_masks(a, fld(bank, F_MOFF))
    a.read_slot(Y, fld(bank, F_B))
    a.idx_on(fld(bank, F_A), mode + ",DST")
    emit()
    if mask:
        a("s_waitcnt lgkmcnt(0)")
        a("s_set_gpr_idx_mode gpr_idx(SRC0,DST)")
        for j in range(8):
            a("v_and_b32_e64 %s, %s, %s" % (v(F[j]), v(F[j]), s(S_M + j)))
    if root:
        a("s_set_gpr_idx_mode gpr_idx(SRC0)")
        a("v_and_b32 %s, %s, %s" % (OP_ROOT, v(F[0]), OP_ROOT))
    a.idx_off()
    dispatch(a, 1 - bank)


def h_add(a, bank, root, mask, dc=False, w32=False, ip=False):
    if ip:
        def emit():
            a("v_add_co_u32 %s, vcc, %s, %s" % (v(F[0]), v(F[0]), v(Y[0])))
            for j in range(1, 8):
                a("v_addc_co_u32 %s, vcc, %s, %s, vcc" % (v(F[j]), v(F[j]), v(Y[j])))
        return inplace_op(a, bank, root, mask, "SRC0", emit)
    if w32:
        return narrow_binop(a, bank, root, mask, dc, "v_add_u32")
    def emit():
        a("v_add_co_u32 %s, vcc, %s, %s" % (v(R[0]), v(F[0]), v(Y[0])))
        for j in range(1, 8):
            a("v_addc_co_u32 %s, vcc, %s, %s, vcc" % (v(R[j]), v(F[j]), v(Y[j])))
    _binop(a, bank, root, mask, emit)


def h_sub(a, bank, root, mask, dc=False, w32=False, ip=False):
    if ip:
        def emit():
            a("v_sub_co_u32 %s, vcc, %s, %s" % (v(F[0]), v(F[0]), v(Y[0])))
            for j in range(1, 8):
                a("v_subb_co_u32 %s, vcc, %s, %s, vcc" % (v(F[j]), v(F[j]), v(Y[j])))
        return inplace_op(a, bank, root, mask, "SRC0", emit)
    if w32:
        return narrow_binop(a, bank, root, mask, dc, "v_sub_u32")
    def emit():
        a("v_sub_co_u32 %s, vcc, %s, %s" % (v(R[0]), v(F[0]), v(Y[0])))
        for j in range(1, 8):
            a("v_subb_co_u32 %s, vcc, %s, %s, vcc" % (v(R[j]), v(F[j]), v(Y[j])))
    _binop(a, bank, root, mask, emit)


def _logic(opname):
    def h(a, bank, root, mask, dc=False, w32=False, ip=False):
        if w32:
            return narrow_binop(a, bank, root, False, dc, opname)
        if ip:
            def emit():
                for j in range(8):
                    a("%s %s, %s, %s" % (opname, v(F[j]), v(F[j]), v(Y[j])))
            return inplace_op(a, bank, root, False, "SRC0", emit)
        def emit():
            for j in range(8):
                a("%s %s, %s, %s" % (opname, v(R[j]), v(F[j]), v(Y[j])))
        _binop(a, bank, root, False, emit)       # canonical in -> canonical out
    return h


h_and = _logic("v_and_b32")
h_or = _logic("v_or_b32")
h_xor = _logic("v_xor_b32")


def h_not(a, bank, root, mask, dc=False, w32=False, ip=False):
    prologue(a, bank)
    if mask:
        load_masks(a, fld(bank, F_MOFF))
    if ip:
        a.idx_on(fld(bank, F_A), "SRC0,DST")
        if mask:
            a("s_waitcnt lgkmcnt(0)")
            for j in range(8):
                a("v_not_b32 %s, %s" % (v(F[j]), v(F[j])))
                a("v_and_b32_e64 %s, %s, %s" % (v(F[j]), v(F[j]), s(S_M + j)))
        else:
            for j in range(8):
                a("v_not_b32 %s, %s" % (v(F[j]), v(F[j])))
        if root:
            a("s_set_gpr_idx_mode gpr_idx(SRC0)")
            a("v_and_b32 %s, %s, %s" % (OP_ROOT, v(F[0]), OP_ROOT))
        a.idx_off()
        return dispatch(a, 1 - bank)
    if w32:
        a.idx_on(fld(bank, F_A), "SRC0")
        a("v_not_b32 %s, %s" % (v(R[0]), v(F[0])))
        a.idx_off()
        return finish_narrow(a, bank, root, mask, dc)
    a.idx_on(fld(bank, F_A), "SRC0")
    for j in range(8):
        a("v_not_b32 %s, %s" % (v(R[j]), v(F[j])))
    a.idx_off()
    finish(a, bank, R, root, mask)


def h_neg(a, bank, root, mask, dc=False, w32=False, ip=False):
    prologue(a, bank)
    if mask:
        load_masks(a, fld(bank, F_MOFF))
    if ip:
        a.idx_on(fld(bank, F_A), "SRC1,DST")
        a("v_sub_co_u32 %s, vcc, 0, %s" % (v(F[0]), v(F[0])))
        for j in range(1, 8):
            a("v_subb_co_u32 %s, vcc, 0, %s, vcc" % (v(F[j]), v(F[j])))
        if mask:
            a("s_waitcnt lgkmcnt(0)")
            a("s_set_gpr_idx_mode gpr_idx(SRC0,DST)")
            for j in range(8):
                a("v_and_b32_e64 %s, %s, %s" % (v(F[j]), v(F[j]), s(S_M + j)))
        if root:
            a("s_set_gpr_idx_mode gpr_idx(SRC0)")
            a("v_and_b32 %s, %s, %s" % (OP_ROOT, v(F[0]), OP_ROOT))
        a.idx_off()
        return dispatch(a, 1 - bank)
    if w32:
        a.idx_on(fld(bank, F_A), "SRC1")
        a("v_sub_u32 %s, 0, %s" % (v(R[0]), v(F[0])))
        a.idx_off()
        return finish_narrow(a, bank, root, mask, dc)
    a.idx_on(fld(bank, F_A), "SRC1")
    a("v_sub_co_u32 %s, vcc, 0, %s" % (v(R[0]), v(F[0])))
    for j in range(1, 8):
        a("v_subb_co_u32 %s, vcc, 0, %s, vcc" % (v(R[j]), v(F[j])))
    a.idx_off()
    finish(a, bank, R, root, mask)


def h_mov(a, bank, root, mask, dc=False, w32=False, ip=False):
    prologue(a, bank)
    if w32:
        a.idx_on(fld(bank, F_A), "SRC0")
        a("v_mov_b32 %s, %s" % (v(R[0]), v(F[0])))
        a.idx_off()
        return finish_narrow(a, bank, root, False, dc)
    a.read_slot(R, fld(bank, F_A))
    finish(a, bank, R, root, False)


def h_root(a, bank, root, mask, dc=False, w32=False, ip=False):
    prologue(a, bank)
    a.idx_on(fld(bank, F_A), "SRC0")
    a("v_and_b32 %s, %s, %s" % (OP_ROOT, v(F[0]), OP_ROOT))
    a.idx_off()
    dispatch(a, 1 - bank)


def _bool_result(a, bank, root, true_if_vcc=True, dc=False):
    if a.nw:                          # dead ROOT-fused Bool: root &= result
        if true_if_vcc:
            a("v_cndmask_b32_e64 %s, 0, %s, vcc" % (OP_ROOT, OP_ROOT))
        else:
            a("v_cndmask_b32_e64 %s, %s, 0, vcc" % (OP_ROOT, OP_ROOT))
        dispatch(a, 1 - bank)
        return
    a("v_cndmask_b32 %s, %s, %s, vcc" % (v(R[0]), "0" if true_if_vcc else "1",
                                         "1" if true_if_vcc else "0"))
    write_narrow(a, bank, v(R[0]), dc)
    if root:
        a.root_and(v(R[0]))
    dispatch(a, 1 - bank)


def _narrow_cmp(a, bank, root, dc, cmp):
    """Bool = cmp(F[a].limb0, F[b].limb0) for operands of at most 32 bits."""
    prologue(a, bank)
    a.idx_on(fld(bank, F_B), "SRC0")
    a("v_mov_b32 %s, %s" % (v(Y[0]), v(F[0])))
    a("s_set_gpr_idx_idx %s" % s(fld(bank, F_A)))
    a("%s vcc, %s, %s" % (cmp, v(F[0]), v(Y[0])))
    a.idx_off()
    _bool_result(a, bank, root, dc=dc)


def h_eq(a, bank, root, mask, dc=False, w32=False, ip=False):
    if w32:
        return _narrow_cmp(a, bank, root, dc, "v_cmp_eq_u32")
    prologue(a, bank)
    a.read_slot(Y, fld(bank, F_B))
    a.idx_on(fld(bank, F_A), "SRC0")
    for j in range(0, 8, 2):        # 64-bit compares (full rate), AND-ed in SALU
        a("v_cmp_eq_u64_e64 %s, %s, %s" % (sp(S_T + j), vp(F[j]), vp(Y[j])))
    a.idx_off()
    a("s_and_b64 %s, %s, %s" % (sp(S_T), sp(S_T), sp(S_T + 2)))
    a("s_and_b64 %s, %s, %s" % (sp(S_T + 4), sp(S_T + 4), sp(S_T + 6)))
    a("s_and_b64 vcc, %s, %s" % (sp(S_T), sp(S_T + 4)))
    _bool_result(a, bank, root, dc=dc)


def _borrow(a, bank, lhs_field, rhs_field):
    """vcc = borrow of F[lhs] - F[rhs] (unsigned lhs < rhs)."""
    a.read_slot(Y, fld(bank, rhs_field))
    a.idx_on(fld(bank, lhs_field), "SRC0")
    a("v_sub_co_u32 %s, vcc, %s, %s" % (v(Y[0]), v(F[0]), v(Y[0])))
    for j in range(1, 8):
        a("v_subb_co_u32 %s, vcc, %s, %s, vcc" % (v(Y[j]), v(F[j]), v(Y[j])))
    a.idx_off()


def h_ult(a, bank, root, mask, dc=False, w32=False, ip=False):
    if w32:
        return _narrow_cmp(a, bank, root, dc, "v_cmp_lt_u32")
    prologue(a, bank)
    _borrow(a, bank, F_A, F_B)
    _bool_result(a, bank, root, dc=dc)


def h_ule(a, bank, root, mask, dc=False, w32=False, ip=False):
    if w32:
        return _narrow_cmp(a, bank, root, dc, "v_cmp_le_u32")
    prologue(a, bank)
    _borrow(a, bank, F_B, F_A)            # b < a  ->  not (a <= b)
    _bool_result(a, bank, root, true_if_vcc=False, dc=dc)


def _scmp(a, bank, root, mask, le: bool, dc: bool = False):
    prologue(a, bank)
    if mask:
        load_masks(a, fld(bank, F_MOFF))
    a.read_slot(X, fld(bank, F_A))
    a.read_slot(Y, fld(bank, F_B))
    if mask:
        a("s_waitcnt lgkmcnt(0)")
        sext(a, X, fld(bank, F_W), S_M, T[0], S_T)
        sext(a, Y, fld(bank, F_W), S_M, T[0], S_T)
    a("v_xor_b32 %s, 0x80000000, %s" % (v(X[7]), v(X[7])))
    a("v_xor_b32 %s, 0x80000000, %s" % (v(Y[7]), v(Y[7])))
    lhs, rhs = (Y, X) if le else (X, Y)
    a("v_sub_co_u32 %s, vcc, %s, %s" % (v(T[0]), v(lhs[0]), v(rhs[0])))
    for j in range(1, 8):
        a("v_subb_co_u32 %s, vcc, %s, %s, vcc" % (v(T[0]), v(lhs[j]), v(rhs[j])))
    _bool_result(a, bank, root, true_if_vcc=not le, dc=dc)


def h_slt(a, bank, root, mask, dc=False, w32=False, ip=False):
    _scmp(a, bank, root, mask, False, dc)


def h_sle(a, bank, root, mask, dc=False, w32=False, ip=False):
    _scmp(a, bank, root, mask, True, dc)


def h_subr(a, bank, root, mask, dc=False, w32=False, ip=False):
    """b - a.  In place on a: F[a] = Y(b) - F[a] (v_subrev)."""
    if ip:
        def emit():
            a("v_subrev_co_u32 %s, vcc, %s, %s" % (v(F[0]), v(F[0]), v(Y[0])))
            for j in range(1, 8):
                a("v_subbrev_co_u32 %s, vcc, %s, %s, vcc" % (v(F[j]), v(F[j]), v(Y[j])))
        return inplace_op(a, bank, root, mask, "SRC0", emit)
    prologue(a, bank)
    if mask:
        load_masks(a, fld(bank, F_MOFF))
    a.read_slot(Y, fld(bank, F_B))
    a.idx_on(fld(bank, F_A), "SRC0")
    a("v_subrev_co_u32 %s, vcc, %s, %s" % (v(R[0]), v(F[0]), v(Y[0])))
    for j in range(1, 8):
        a("v_subbrev_co_u32 %s, vcc, %s, %s, vcc" % (v(R[j]), v(F[j]), v(Y[j])))
    a.idx_off()
    finish(a, bank, R, root, mask)


def _ite_cond(a: Asm, bank: int, negate: bool):
    """vcc = (c != 0), or (c == 0) when negated; c is a canonical Bool
    (limb 0 is 0 or 1), compared straight from the file."""
    a.idx_on(fld(bank, F_C), "SRC0")
    a("v_cmp_%s_u32_e64 vcc, %s, 0" % ("eq" if negate else "ne", v(F[0])))
    a.idx_off()


def _ite_inplace(a: Asm, bank: int, root: bool, negate: bool):
    """F[a] = cond ? F[a] : F[b]   (ITE, dest == a)
       F[a] = cond ? F[b] : F[a]   (ITEN, dest == a): vcc = !cond.
    F[b] is copied in the lanes that select it (under exec)."""
    prologue(a, bank)
    _ite_cond(a, bank, not negate)           # vcc set where F[b] is selected
    a.read_slot(Y, fld(bank, F_B))
    lab = exec_begin(a, None, S_T)
    a.idx_on(fld(bank, F_A), "DST")
    moves(a, F, Y)
    a.idx_off()
    exec_end(a, lab, S_T)
    if root:
        a.idx_on(fld(bank, F_A), "SRC0")
        a("v_and_b32 %s, %s, %s" % (OP_ROOT, v(F[0]), OP_ROOT))
        a.idx_off()
    dispatch(a, 1 - bank)


def _ite_select(a: Asm, bank: int, first: int, other: int):
    """R = F[first], then F[other] read straight into R in the lanes where
    vcc is set (an indexed read under exec: no staging copy)."""
    a.read_slot(R, fld(bank, first))
    lab = exec_begin(a, None, S_T)
    a.read_slot(R, fld(bank, other))
    exec_end(a, lab, S_T)


def h_iten(a, bank, root, mask, dc=False, w32=False, ip=False):
    """c ? b : a."""
    if ip:
        return _ite_inplace(a, bank, root, True)
    prologue(a, bank)
    _ite_cond(a, bank, False)                # vcc = c: take F[b]
    _ite_select(a, bank, F_A, F_B)
    finish(a, bank, R, root, False)


def h_ite(a, bank, root, mask, dc=False, w32=False, ip=False):
    if ip:
        return _ite_inplace(a, bank, root, False)
    prologue(a, bank)
    if w32:
        _ite_cond(a, bank, False)
        a.idx_on(fld(bank, F_B), "SRC0")
        a("v_mov_b32 %s, %s" % (v(Y[0]), v(F[0])))
        a("s_set_gpr_idx_idx %s" % s(fld(bank, F_A)))
        a("s_set_gpr_idx_mode gpr_idx(SRC1)")
        a("v_cndmask_b32 %s, %s, %s, vcc" % (v(R[0]), v(Y[0]), v(F[0])))
        a.idx_off()
        return finish_narrow(a, bank, root, False, dc)
    _ite_cond(a, bank, True)                 # vcc = !c: take F[b]
    _ite_select(a, bank, F_A, F_B)
    finish(a, bank, R, root, False)


def h_extract(a, bank, root, mask, dc=False, w32=False, ip=False):
    """R = (F[a] >> lo) & mask(W).  C = 8a + (lo >> 5) + 8, IMM = lo & 31."""
    prologue(a, bank)
    load_masks(a, fld(bank, F_MOFF))
    if w32:
        a.idx_on(fld(bank, F_C), "SRC0,SRC1")
        a("v_alignbit_b32 %s, %s, %s, %s" % (v(R[0]), v(G[1]), v(G[0]), s(fld(bank, F_IMM))))
        a.idx_off()
        return finish_narrow(a, bank, root, True, dc)
    a.idx_on(fld(bank, F_C), "SRC0,SRC1")
    for j in range(8):
        a("v_alignbit_b32 %s, %s, %s, %s" % (v(R[j]), v(G[j + 1]), v(G[j]), s(fld(bank, F_IMM))))
    a.idx_off()
    finish(a, bank, R, root, True)


def h_concat(a, bank, root, mask, dc=False, w32=False, ip=False):
    """R = F[a] << sb | F[b] (sb = width of b).  C = funnel index, IMM =
    funnel shift; MOFF -> 8 masks of the bits >= sb."""
    prologue(a, bank)
    load_masks(a, fld(bank, F_MOFF))
    a.read_slot(Y, fld(bank, F_B))
    a.idx_on(fld(bank, F_C), "SRC0,SRC1")
    for j in range(8):
        a("v_alignbit_b32 %s, %s, %s, %s" % (v(R[j]), v(G[j + 1]), v(G[j]), s(fld(bank, F_IMM))))
    a.idx_off()
    a("s_waitcnt lgkmcnt(0)")
    for j in range(8):
        a("v_bfi_b32 %s, %s, %s, %s" % (v(R[j]), s(S_M + j), v(R[j]), v(Y[j])))
    finish(a, bank, R, root, False)


def h_extractn(a: Asm, bank: int, var: int):
    """EXTRACT to W > 32 bits with nl = var + 1 result limbs known
    statically: nl funnel shifts, the top limb masked with the value in MOFF
    (bits < W mod 32, all ones when W is a multiple of 32), zero limbs
    above, written as pairs."""
    nl = var + 1
    prologue(a, bank)
    a.idx_on(fld(bank, F_C), "SRC0,SRC1")
    for j in range(nl):
        a("v_alignbit_b32 %s, %s, %s, %s" % (v(R[j]), v(G[j + 1]), v(G[j]), s(fld(bank, F_IMM))))
    a.idx_off()
    a("v_and_b32 %s, %s, %s" % (v(R[nl - 1]), s(fld(bank, F_MOFF)), v(R[nl - 1])))
    a.idx_on(fld(bank, F_D), "DST")
    moves(a, F, [R[j] if j < nl else None for j in range(8)])
    a.idx_off()
    dispatch(a, 1 - bank)


def h_concatq(a: Asm, bank: int, var: int):
    """CONCAT R = F[a] << k | F[b] with q = k >> 5 (var & 7) and a bit shift
    k & 31 (var & 8) known statically: limbs below q come from F[b], limbs
    from q up from the funnel shift of F[a] (C = funnel index, IMM = funnel
    shift), limb q merged with MOFF = the bits >= k & 31; written as pairs."""
    q, bs = var & 7, bool(var & 8)
    ny = q + (1 if bs else 0)                 # limbs of F[b] needed
    prologue(a, bank)
    if ny:
        a.idx_on(fld(bank, F_B), "SRC0")
        for j in range(0, ny, 2):
            a("v_mov_b64 %s, %s" % (vp(Y[j]), vp(F[j])))
        a.idx_off()
    a.idx_on(fld(bank, F_C), "SRC0,SRC1")
    for j in range(q, 8):
        a("v_alignbit_b32 %s, %s, %s, %s" % (v(R[j]), v(G[j + 1]), v(G[j]), s(fld(bank, F_IMM))))
    a.idx_off()
    if bs:
        a("v_bfi_b32 %s, %s, %s, %s" % (v(R[q]), s(fld(bank, F_MOFF)), v(R[q]), v(Y[q])))
    a.idx_on(fld(bank, F_D), "DST")
    moves(a, F, [Y[j] if j < q else R[j] for j in range(8)])
    a.idx_off()
    dispatch(a, 1 - bank)


def h_sext(a, bank, root, mask, dc=False, w32=False, ip=False):
    """sign_extend from IMM bits to W bits.  MOFF -> 16 masks: bits < IMM,
    then bits < W."""
    prologue(a, bank)
    load_masks(a, fld(bank, F_MOFF))
    a("s_add_u32 %s, %s, 32" % (s(S_T), s(fld(bank, F_MOFF))))
    a("s_load_dwordx8 s[%d:%d], %s, %s" % (S_CUR, S_CUR + 7, sp(S_CONST), s(S_T)))
    a.read_slot(R, fld(bank, F_A))
    a("s_waitcnt lgkmcnt(0)")
    sext(a, R, fld(bank, F_IMM), S_M, T[0], S_T)
    a.write_slot(R, fld(bank, F_D), S_CUR)
    if root:
        a.root_and(v(R[0]))
    dispatch(a, 1 - bank)


def h_spill_lds(a: Asm, bank: int, var: int):
    """LDS spill straight from slot ``var & 15``; NARROW: a one-limb value,
    one dword at the record's dword position of its region (the translator
    packs one-limb values eight to a region, mg_host.cpp place_spills)."""
    fa = FB + 8 * (var & 15)
    prologue(a, bank)
    if JIT:       # the halves' byte offsets are the record's: instruction offsets
        if var & V_NARROW:
            a("ds_write_b32 %s, v%d offset:@F%d@" % (OP_LDS, fa, F_IMM))
            return dispatch(a, 1 - bank)
        a("ds_write_b128 %s, v[%d:%d] offset:@F%d@" % (OP_LDS, fa, fa + 3, F_IMM))
        a("ds_write_b128 %s, v[%d:%d] offset:@F%d@" % (OP_LDS, fa + 4, fa + 7, F_MOFF))
        return dispatch(a, 1 - bank)
    a("v_add_u32 %s, %s, %s" % (v(T[0]), s(fld(bank, F_IMM)), OP_LDS))
    if var & V_NARROW:
        a("ds_write_b32 %s, v%d" % (v(T[0]), fa))
        return dispatch(a, 1 - bank)
    a("v_add_u32 %s, %s, %s" % (v(T[1]), s(fld(bank, F_MOFF)), OP_LDS))
    a("ds_write_b128 %s, v[%d:%d]" % (v(T[0]), fa, fa + 3))
    a("ds_write_b128 %s, v[%d:%d]" % (v(T[1]), fa + 4, fa + 7))
    dispatch(a, 1 - bank)


def h_reload_lds(a: Asm, bank: int, var: int):
    """LDS reload straight into slot ``var & 15``; the dispatch's lgkmcnt wait
    covers the reads.  NARROW: one dword, limbs 1..7 zeroed."""
    fd = FB + 8 * (var & 15)
    prologue(a, bank)
    if JIT:
        lo, hi = (OP_LDS, " offset:@F%d@" % F_IMM), (OP_LDS, " offset:@F%d@" % F_MOFF)
    else:
        a("v_add_u32 %s, %s, %s" % (v(T[0]), s(fld(bank, F_IMM)), OP_LDS))
        lo = hi = (v(T[0]), "")
        if not var & V_NARROW:
            a("v_add_u32 %s, %s, %s" % (v(T[1]), s(fld(bank, F_MOFF)), OP_LDS))
            hi = (v(T[1]), "")
    if var & V_NARROW:
        a("ds_read_b32 v%d, %s%s" % ((fd,) + lo))
        moves(a, [fd + j for j in range(1, 8)], [None] * 7)
        return dispatch(a, 1 - bank)
    a("ds_read_b128 v[%d:%d], %s%s" % ((fd, fd + 3) + lo))
    a("ds_read_b128 v[%d:%d], %s%s" % ((fd + 4, fd + 7) + hi))
    dispatch(a, 1 - bank)


def h_spill_scr(a: Asm, bank: int, var: int):
    """Scratch spill straight from slot ``var & 15``; NARROW: a one-limb
    value, one dword (its RELOADD zeroes limbs 1..7)."""
    fa = FB + 8 * (var & 15)
    prologue(a, bank)
    a("s_add_u32 %s, %s, %s" % (s(S_T), IN["scr"], s(fld(bank, F_IMM))))
    if var & V_NARROW:
        a("scratch_store_dword off, v%d, %s" % (fa, s(S_T)))
    else:
        a("scratch_store_dwordx4 off, v[%d:%d], %s" % (fa, fa + 3, s(S_T)))
        a("scratch_store_dwordx4 off, v[%d:%d], %s offset:16" % (fa + 4, fa + 7, s(S_T)))
    dispatch(a, 1 - bank)


def h_reload_scr(a, bank, root, mask, dc=False, w32=False, ip=False):
    prologue(a, bank)
    a("s_add_u32 %s, %s, %s" % (s(S_T), IN["scr"], s(fld(bank, F_IMM))))
    a("scratch_load_dwordx4 v[%d:%d], off, %s" % (R[0], R[3], s(S_T)))
    a("scratch_load_dwordx4 v[%d:%d], off, %s offset:16" % (R[4], R[7], s(S_T)))
    a("s_waitcnt vmcnt(0)")
    finish(a, bank, R, root, False)


def _soa_base(a: Asm, ptr_op: str, row_sgpr: int):
    """s[S_T:S_T+1] = ptr + (8*index) * stride*4 ; s[S_T+4:S_T+5] = stride*4.
    Clobbers S_T..S_T+5."""
    a("s_lshl_b64 %s, %s, 2" % (sp(S_T + 4), IN["stride"]))
    a("s_lshl_b32 %s, %s, 3" % (s(S_T + 1), s(row_sgpr)))
    a("s_mul_i32 %s, %s, %s" % (s(S_T), s(S_T + 1), s(S_T + 4)))
    a("s_mul_hi_u32 %s, %s, %s" % (s(S_T + 2), s(S_T + 1), s(S_T + 4)))
    a("s_mul_i32 %s, %s, %s" % (s(S_T + 3), s(S_T + 1), s(S_T + 5)))
    a("s_add_u32 %s, %s, %s" % (s(S_T + 1), s(S_T + 2), s(S_T + 3)))
    a("s_mov_b64 %s, %s" % (sp(S_T + 2), ptr_op))
    a("s_add_u32 %s, %s, %s" % (s(S_T), s(S_T), s(S_T + 2)))
    a("s_addc_u32 %s, %s, %s" % (s(S_T + 1), s(S_T + 1), s(S_T + 3)))


def lane_offset(a: Asm, dst: int):
    """v[dst] = 4 * lane (the lane's row in an SoA buffer) from idx - first.
    Clobbers s[S_T+6:S_T+7]."""
    a("s_mov_b64 %s, %s" % (sp(S_T + 6), IN["first"]))
    a("v_subrev_u32 %s, %s, %s" % (v(dst), s(S_T + 6), OP_IDX_LO))
    a("v_lshlrev_b32 %s, 2, %s" % (v(dst), v(dst)))


def _soa_step(a: Asm):
    a("s_add_u32 %s, %s, %s" % (s(S_T), s(S_T), s(S_T + 4)))
    a("s_addc_u32 %s, %s, %s" % (s(S_T + 1), s(S_T + 1), s(S_T + 5)))


def _store_soa(a: Asm, regs: List[int], ptr_op: str, row_sgpr: int, wait_vm: bool = False,
               cold: bool = False):
    """regs -> SoA buffer ptr[(8*row + j) * stride + lane], active lanes only,
    when ptr != 0 (after the in-flight loads into regs with wait_vm); with
    ``cold`` the store is out of line (the caller flushes it) and the
    ptr == 0 case runs straight through.  Clobbers S_T..S_T+7, T[0]."""
    skip = a.uniq("nost")
    a("s_cmp_lg_u64 %s, 0" % ptr_op)
    if cold:
        lab = a.uniq("sst")
        a("s_cbranch_scc1 %s" % lab)
        a.label(skip)
        a.cold()
        a.label(lab)
        _store_soa_body(a, regs, ptr_op, row_sgpr, wait_vm)
        a("s_branch %s" % skip)
        a.hot()
        return
    a("s_cbranch_scc0 %s" % skip)
    _store_soa_body(a, regs, ptr_op, row_sgpr, wait_vm)
    a.label(skip)


def _store_soa_body(a: Asm, regs: List[int], ptr_op: str, row_sgpr: int, wait_vm: bool):
    if wait_vm:
        a("s_waitcnt vmcnt(0)")
    _soa_base(a, ptr_op, row_sgpr)
    lane_offset(a, T[0])
    a("s_mov_b64 %s, exec" % sp(S_T + 6))
    a("s_mov_b64 exec, %s" % IN["active"])
    for j in range(8):
        a("global_store_dword %s, %s, %s" % (v(T[0]), v(regs[j]), sp(S_T)))
        if j < 7:
            _soa_step(a)
    a("s_mov_b64 exec, %s" % sp(S_T + 6))


def h_out(a, bank, root, mask, dc=False, w32=False, ip=False):
    """probe[C] = F[a] (active lanes, when a probe buffer is bound)."""
    prologue(a, bank)
    a.read_slot(Y, fld(bank, F_A))
    _store_soa(a, Y, IN["probes"], fld(bank, F_C))
    dispatch(a, 1 - bank)


# ---------------------------------------------------------------------------
# LEAF: eval mode (SoA load) or the device candidate generator
# ---------------------------------------------------------------------------

GOLD = 0x9E3779B97F4A7C15
MIX1 = 0xBF58476D1CE4E5B9                         # the one 64-bit multiplier (generator v9)
PAIR_MUL = (0x85EBCA6B, 0xC2B2AE35, 0x27D4EB2F)   # uniform limb pairs 1-3 (generator v6)
CLS_MUL = 0x2545F491                              # class remix (generator v7/v8)
# mixer constants live in SGPRs s[S_K:S_K+5], set once at entry
K_GOLD_LO, K_GOLD_HI, K_M1_LO, K_M1_HI, K_M2_LO, K_M2_HI = range(S_K, S_K + 6)
S_GROUP = K_GOLD_LO        # compiled programs: lo32(idx >> 6) of the wave (jit.program_asm)
S_PAIR = S_X + 2           # s[90:92] the uniform limb-pair multipliers during a LEAF


def load_sm64_consts(a: Asm):
    # (GOLD goes in as literals; s[96:97] hold a compiled program's wave
    # group, S_GROUP, set at the program's entry)
    # (v9's single multiplier frees s[100:101]: two uniform-limb multipliers)
    consts = [(K_M1_LO, MIX1), (K_M1_HI, MIX1 >> 32),
              (K_M2_LO, PAIR_MUL[0]), (K_M2_HI, PAIR_MUL[1])]
    for reg, val in consts:
        a("s_mov_b32 %s, 0x%x" % (s(reg), val & 0xFFFFFFFF))


def sm64(a: Asm, st: List[int], z: List[int], t: List[int]):
    """The candidate mixer (generator v9) on the per-lane state st = (lo,
    hi): st += GOLD; u = st ^ (st >> 32); z = u * MIX1 (mod 2^64); r0 =
    z ^ (z >> 32).  Every step is a bijection of 64-bit words, so distinct
    candidate indices give distinct r0 per leaf.  v8 ran SplitMix64's
    finaliser (three 64-bit xorshifts, two 64-bit multiplies: 19 VALU); the
    32-bit-aligned xorshifts are one v_xor each and one multiply stays
    (8 VALU).  Constants in SGPRs (load_sm64_consts); t: 4 temps with
    t[0]:t[1] and t[2]:t[3] aligned; t[3] holds GOLD_HI on entry (set once
    per leaf; read as the don't-care high half of the cross-term addend).
    Uses vcc (also as the mads' junk carry-out)."""
    a("v_add_co_u32 %s, vcc, 0x%x, %s" % (v(st[0]), GOLD & 0xFFFFFFFF, v(st[0])))
    a("v_addc_co_u32 %s, vcc, %s, %s, vcc" % (v(st[1]), v(t[3]), v(st[1])))
    a("v_xor_b32 %s, %s, %s" % (v(z[0]), v(st[0]), v(st[1])))                    # u_lo
    # z = u * MIX1 with u = (z[0], st[1]): the two cross terms' low word
    # (lo * K_hi by v_mul_lo, hi * K_lo + it by the low half of a mad), the
    # full low product by a mad, the cross word added to its high half
    a("v_mul_lo_u32 %s, %s, %s" % (v(t[2]), v(z[0]), s(K_M1_HI)))
    a("v_mad_u64_u32 %s, vcc, %s, %s, %s" % (vp(t[0]), v(st[1]), s(K_M1_LO), vp(t[2])))
    a("v_mad_u64_u32 %s, vcc, %s, %s, 0" % (vp(z[0]), v(z[0]), s(K_M1_LO)))
    a("v_add_u32 %s, %s, %s" % (v(z[1]), v(z[1]), v(t[0])))
    a("v_xor_b32 %s, %s, %s" % (v(z[0]), v(z[0]), v(z[1])))                       # r0_lo


def _uniform_limbs(a: Asm, dst: List[int], z: List[int], x: int):
    """The uniform class's value: r0 in limbs 0-1, limb pair k = 1..3 is
    x * C_k + r0 (mod 2^64) with x = lo ^ hi of r0 — one v_mad_u64_u32 per
    two limbs (v6; v4 spent a 4-VALU multiply-xorshift per limb).  Uses
    s[S_PAIR..S_PAIR+2] and v[x]."""
    if dst[0] != z[0]:
        a("v_mov_b64 %s, %s" % (vp(dst[0]), vp(z[0])))
    a("v_xor_b32 %s, %s, %s" % (v(x), v(z[0]), v(z[1])))
    # v9: the first two multipliers are resident in s[100:101] (set at entry)
    regs = [K_M2_LO, K_M2_HI, S_PAIR + 2]
    a("s_mov_b32 %s, 0x%x" % (s(regs[2]), PAIR_MUL[2]))
    for k in range(3):
        a("v_mad_u64_u32 %s, vcc, %s, %s, %s" % (vp(dst[2 + 2 * k]), v(x), s(regs[k]),
                                                 vp(z[0])))


def _boundary_loads(a: Asm, dst: List[int], lo: int, f, tt: List[int]):
    """Boundary values {0, 1, 2^(w-1), 2^256-1, 2^k+1, 2^k-1}: one load pair
    from the context's boundary table (mg_api.cpp mg_boundary_table): entry
    kind * 256 + p, p = w - 1 for kind 2 and k otherwise, kind = mulhi(lo,
    6), k = mulhi(lo * 0x9E3779B1, w); masked to the width by the handler.
    The table pointer is loaded here, into s[S_T+6:S_T+7] (only waves of
    this class pay for it; that pair is the dispatch's jump target, so the
    load is settled before the block ends)."""
    a("s_load_dwordx2 %s, %s, 0x38" % (sp(S_T + 6), IN["desc"]))   # boundary table
    kind, k, bit = tt[0], tt[1], tt[2]
    a("v_mul_hi_u32 %s, %s, 6" % (v(kind), v(lo)))
    a("s_mov_b32 %s, 0x9e3779b1" % s(S_T))
    a("v_mul_lo_u32 %s, %s, %s" % (v(k), v(lo), s(S_T)))
    a("v_mul_hi_u32 %s, %s, %s" % (v(k), v(k), s(f["w"])))
    a("s_sub_u32 %s, %s, 1" % (s(S_T + 1), s(f["w"])))
    a("v_mov_b32 %s, %s" % (v(bit), s(S_T + 1)))
    a("v_cmp_eq_u32 vcc, 2, %s" % v(kind))
    a("v_cndmask_b32 %s, %s, %s, vcc" % (v(k), v(k), v(bit)))
    a("v_lshl_add_u32 %s, %s, 8, %s" % (v(k), v(kind), v(k)))
    a("v_lshlrev_b32 %s, 5, %s" % (v(k), v(k)))
    a("s_waitcnt lgkmcnt(0)")
    a("global_load_dwordx4 v[%d:%d], %s, %s" % (dst[0], dst[3], v(k), sp(S_T + 6)))
    a("global_load_dwordx4 v[%d:%d], %s, %s offset:16" % (dst[4], dst[7], v(k), sp(S_T + 6)))


def _pool_loads(a: Asm, dst: List[int], lo: int, f, tt: List[int]):
    """Pool values consts[pool_off + e] + delta - 1, stored as (v-1, v, v+1)
    triples (entry e * 3 + delta): e = mulhi(lo, pool_n), delta =
    mulhi(lo * 0x85EBCA6B, 3); one load pair."""
    e, delta = tt[0], tt[1]
    a("v_mul_hi_u32 %s, %s, %s" % (v(e), v(lo), s(f["pn"])))
    a("s_mov_b32 %s, 0x85ebca6b" % s(S_T))
    a("v_mul_lo_u32 %s, %s, %s" % (v(delta), v(lo), s(S_T)))
    a("v_mul_hi_u32 %s, %s, 3" % (v(delta), v(delta)))
    a("v_mad_u32_u24 %s, %s, 3, %s" % (v(e), v(e), v(delta)))
    a("v_lshl_add_u32 %s, %s, 5, %s" % (v(e), v(e), s(f["poff"])))
    a("global_load_dwordx4 v[%d:%d], %s, %s" % (dst[0], dst[3], v(e), sp(S_CONST)))
    a("global_load_dwordx4 v[%d:%d], %s, %s offset:16" % (dst[4], dst[7], v(e), sp(S_CONST)))


def _gen_leaf(a: Asm, bank: int, dst: Optional[List[int]] = None, wait: bool = True,
              nested: bool = False, aligned: bool = False):
    """dst[0..7] (default X) <- generator value of leaf C for candidate
    first + lane; the boundary / pool lanes arrive by loads into dst, waited
    for unless wait=False (LEAFD: the translator places the WAITVM).
    Mirrors oracle/gen_ref.py gen_leaf (generator v8).  r0 = SplitMix64 of
    the candidate index is computed per lane; the class (v8) is drawn once
    per group of 64 consecutive indices, so when every active lane of the
    wave is in one group — every wave of a launch that starts at a multiple
    of 64: all search and bench launches — the class is wave-uniform and
    only its own code runs (branch on the scalar class, computed in SALU
    from the first active lane's index).  A wave across two groups (an
    unaligned eval) draws per lane and runs the two classes in turn.
    Device descriptor (8 words at gen + 32*leaf): width, pool_off (bytes),
    pool_n, pct_uniform, pct_small, pct_boundary, salt_lo, salt_hi.  A
    LEAFD (``in_record``: 256 bits) finds them in its own record instead
    (mg_load_program: pool_off, salt, pool_n, packed thresholds), so no
    descriptor load sits between dispatch and the generator."""
    in_record = dst is not None and dst != X
    dst = X if dst is None else dst
    # the mixer writes r0 straight into the value's first two limbs (the
    # uniform and small classes keep it there; the load classes read its
    # low word for their address before the loads overwrite it)
    st, z, tt = [T[0], T[1]], [dst[0], dst[1]], [T[4], T[5], T[6], T[7]]
    cls, lo = T[8], z[0]
    g = S_CUR
    flat = JIT

    def record_fields():
        # width and class thresholds from the LEAFD record (in a compiled
        # program they are constants: set after the branches that skip
        # them, they fold into the compares as literals)
        a("s_movk_i32 %s, 0x100" % s(f["w"]))
        pk = fld(bank, LEAFD_PCT)
        a("s_and_b32 %s, %s, 0xff" % (s(f["pu"]), s(pk)))
        a("s_bfe_u32 %s, %s, 0x80008" % (s(f["ps"]), s(pk)))
        a("s_bfe_u32 %s, %s, 0x80010" % (s(f["pb"]), s(pk)))
    if in_record:
        f = {"w": g + 0, "poff": fld(bank, LEAFD_POFF), "pn": fld(bank, LEAFD_PN),
             "pu": g + 3, "ps": g + 4, "pb": g + 5, "salt": fld(bank, LEAFD_SALT)}
        if not flat:
            record_fields()
    else:
        f = {"w": g + 0, "poff": g + 1, "pn": g + 2, "pu": g + 3, "ps": g + 4, "pb": g + 5,
             "salt": g + 6}
        a("s_load_dwordx2 %s, %s, 0x10" % (sp(S_T), IN["desc"]))       # gen table
        a("s_lshl_b32 %s, %s, 5" % (s(S_T + 2), s(fld(bank, F_C))))
        a("s_waitcnt lgkmcnt(0)")
        a("s_load_dwordx8 s[%d:%d], %s, %s" % (g, g + 7, sp(S_T), s(S_T + 2)))
    # st = seed ^ salt ^ idx (v5: the counter itself, SplitMix64's finaliser
    # spreads it; no idx * GOLD multiply); idx = first + lane arrives ready
    a("v_mov_b32 %s, 0x%x" % (v(tt[3]), GOLD >> 32))
    if not in_record:
        a("s_waitcnt lgkmcnt(0)")
    if flat and in_record:                           # ss = seed ^ salt, the salt as literals
        seed = int(PINNED["seed"][2:].split(":")[0])
        a("s_xor_b32 %s, %s, %s" % (s(S_T), s(seed), s(f["salt"])))
        a("s_xor_b32 %s, %s, %s" % (s(S_T + 1), s(seed + 1), s(f["salt"] + 1)))
    else:
        a("s_xor_b64 %s, %s, %s" % (sp(S_T), IN["seed"], sp(f["salt"])))     # ss = seed ^ salt
    a("v_xor_b32 %s, %s, %s" % (v(st[0]), s(S_T), OP_IDX_LO))
    a("v_xor_b32 %s, %s, %s" % (v(st[1]), s(S_T + 1), OP_IDX_HI))
    # v8 class: cls = mulhi(((lo32(idx >> 6) ^ lo32(ss)) * CLS_MUL) ^ hi32(ss), 100)
    # When the first active lane's index is a multiple of 64 every active
    # lane is in its group (a wave's indices are consecutive): the class is
    # computed once, in SALU, from that index.  Otherwise (out of line) per
    # lane, and a waterfall runs each distinct class of the wave in turn:
    # exec = the lanes whose draw equals the first active lane's, that
    # class's code, repeat with the rest (a wave of consecutive indices spans
    # at most two groups).
    sc, rest, save = S_T + 2, S_T + 4, S_X          # (division's lane masks: free here)
    lab_slow, lab_join, lab_loop, lab_again = (a.uniq("gslow"), a.uniq("gjoin"), a.uniq("gcls"),
                                               a.uniq("gagain"))
    lab_disp = a.uniq("gdisp")
    lab_uni, lab_small, lab_bnd, lab_done = (a.uniq("guni"), a.uniq("gsml"), a.uniq("gbnd"),
                                             a.uniq("gdone"))
    def lane_class():
        # per-lane class draws (ss still in s[S_T:S_T+1]); rest != 0 sends
        # the join to the waterfall
        a("v_alignbit_b32 %s, %s, %s, 6" % (v(cls), OP_IDX_HI, OP_IDX_LO))
        a("v_xor_b32 %s, %s, %s" % (v(cls), s(S_T), v(cls)))
        a("s_mov_b32 %s, 0x%x" % (s(sc), CLS_MUL))
        a("v_mul_lo_u32 %s, %s, %s" % (v(cls), v(cls), s(sc)))
        a("v_xor_b32 %s, %s, %s" % (v(cls), s(S_T + 1), v(cls)))
        a("s_movk_i32 %s, 100" % s(sc))
        a("v_mul_hi_u32 %s, %s, %s" % (v(cls), v(cls), s(sc)))
        a("s_mov_b64 %s, -1" % sp(rest))


    def classes(lab_out):
        # the class dispatch on s[sc] and the four classes' code, every exit
        # at lab_out
        l_uni, l_small, l_bnd = a.uniq("guni"), a.uniq("gsml"), a.uniq("gbnd")
        a("s_cmp_lt_u32 %s, %s" % (s(sc), s(f["pu"])))
        a("s_cbranch_scc1 %s" % l_uni)                   # cls < pct_uniform
        a("s_cmp_lt_u32 %s, %s" % (s(sc), s(f["ps"])))
        a("s_cbranch_scc1 %s" % l_small)
        a("s_cmp_lt_u32 %s, %s" % (s(sc), s(f["pb"])))
        a("s_cbranch_scc1 %s" % l_bnd)
        a("s_cmp_eq_u32 %s, 0" % s(f["pn"]))
        a("s_cbranch_scc1 %s" % l_uni)                   # pool class, empty pool
        _pool_loads(a, dst, lo, f, tt)                   # pool
        a("s_branch %s" % lab_out)
        a.label(l_bnd)
        _boundary_loads(a, dst, lo, f, tt)
        a("s_branch %s" % lab_out)
        a.label(l_small)                                 # small: r0 (< 2^64)
        moves(a, dst[2:], [None] * 6)
        a("s_branch %s" % lab_out)
        a.label(l_uni)
        _uniform_limbs(a, dst, z, tt[0])

    if flat and aligned:
        # compiled program, wave known aligned (S_FAST): its group is in
        # s[S_GROUP] since the program's entry — the class is four SALU
        a("s_xor_b32 %s, %s, %s" % (s(sc), s(S_GROUP), s(S_T)))
        a("s_mul_i32 %s, %s, 0x%x" % (s(sc), s(sc), CLS_MUL))
        a("s_xor_b32 %s, %s, %s" % (s(sc), s(sc), s(S_T + 1)))
        a("s_mul_hi_u32 %s, %s, 100" % (s(sc), s(sc)))
        if in_record:
            record_fields()
        sm64(a, st, z, tt)
        classes(lab_done)
        a.label(lab_done)
        if wait:
            a("s_waitcnt vmcnt(0)")                      # boundary and pool loads
        return
    if flat:
        # compiled programs (straight-line, cold code at the program's end):
        # the wave-uniform class runs the dispatch with no waterfall state
        # at all; an unaligned wave takes a cold copy of mixer + dispatch
        # inside its own waterfall
        lab_wdone = a.uniq("gwdone")
        a("v_readfirstlane_b32 %s, %s" % (s(sc), OP_IDX_LO))
        a("v_readfirstlane_b32 %s, %s" % (s(sc + 1), OP_IDX_HI))
        a("s_and_b32 %s, %s, 63" % (s(rest), s(sc)))
        a("s_cbranch_scc1 %s" % lab_slow)
        a("s_lshr_b64 %s, %s, 6" % (sp(sc), sp(sc)))
        a("s_xor_b32 %s, %s, %s" % (s(sc), s(sc), s(S_T)))
        a("s_mul_i32 %s, %s, 0x%x" % (s(sc), s(sc), CLS_MUL))
        a("s_xor_b32 %s, %s, %s" % (s(sc), s(sc), s(S_T + 1)))
        a("s_mul_hi_u32 %s, %s, 100" % (s(sc), s(sc)))
        if in_record:
            record_fields()
        sm64(a, st, z, tt)
        classes(lab_done)
        a.label(lab_done)
        if wait:
            a("s_waitcnt vmcnt(0)")                      # boundary and pool loads
        lab_after = a.uniq("gafter")
        if nested:                                       # already out of line
            a("s_branch %s" % lab_after)
        else:
            a.cold()
        a.label(lab_slow)
        if in_record:
            record_fields()
        lane_class()
        sm64(a, st, z, tt)
        a("s_mov_b64 %s, exec" % sp(save))
        a.label(lab_loop)
        a("v_readfirstlane_b32 %s, %s" % (s(sc), v(cls)))
        a("v_cmp_eq_u32 vcc, %s, %s" % (s(sc), v(cls)))
        a("s_and_saveexec_b64 %s, vcc" % sp(rest))
        a("s_andn2_b64 %s, %s, exec" % (sp(rest), sp(rest)))   # lanes still to do
        classes(lab_wdone)
        a.label(lab_wdone)
        a("s_mov_b64 exec, %s" % sp(rest))
        a("s_cbranch_execnz %s" % lab_again)
        a("s_mov_b64 exec, %s" % sp(save))
        a("s_branch %s" % lab_done)
        # another group in this wave: its loads are in flight into other lanes
        # of dst; settle them before the next class writes dst
        a.label(lab_again)
        a("s_waitcnt vmcnt(0)")
        a("s_branch %s" % lab_loop)
        if nested:
            a.label(lab_after)
        else:
            a.hot()
        return
    a("v_readfirstlane_b32 %s, %s" % (s(sc), OP_IDX_LO))
    a("v_readfirstlane_b32 %s, %s" % (s(sc + 1), OP_IDX_HI))
    a("s_and_b32 %s, %s, 63" % (s(rest), s(sc)))
    a("s_cbranch_scc1 %s" % lab_slow)
    a("s_lshr_b64 %s, %s, 6" % (sp(sc), sp(sc)))
    a("s_xor_b32 %s, %s, %s" % (s(sc), s(sc), s(S_T)))
    a("s_mul_i32 %s, %s, 0x%x" % (s(sc), s(sc), CLS_MUL))
    a("s_xor_b32 %s, %s, %s" % (s(sc), s(sc), s(S_T + 1)))
    a("s_mul_hi_u32 %s, %s, 100" % (s(sc), s(sc)))
    a("s_mov_b64 %s, 0" % sp(rest))                 # one pass: no lanes left after it
    a.label(lab_join)
    sm64(a, st, z, tt)
    a("s_mov_b64 %s, exec" % sp(save))
    a("s_cmp_lg_u64 %s, 0" % sp(rest))
    a("s_cbranch_scc1 %s" % lab_loop)                # per-lane classes: the waterfall
    a.label(lab_disp)
    a("s_cmp_lt_u32 %s, %s" % (s(sc), s(f["pu"])))
    a("s_cbranch_scc1 %s" % lab_uni)                 # cls < pct_uniform
    a("s_cmp_lt_u32 %s, %s" % (s(sc), s(f["ps"])))
    a("s_cbranch_scc1 %s" % lab_small)
    a("s_cmp_lt_u32 %s, %s" % (s(sc), s(f["pb"])))
    a("s_cbranch_scc1 %s" % lab_bnd)
    a("s_cmp_eq_u32 %s, 0" % s(f["pn"]))
    a("s_cbranch_scc1 %s" % lab_uni)                 # pool class, empty pool
    _pool_loads(a, dst, lo, f, tt)                   # pool
    a("s_branch %s" % lab_done)
    a.label(lab_bnd)
    _boundary_loads(a, dst, lo, f, tt)
    a("s_branch %s" % lab_done)
    a.label(lab_small)                               # small: r0 (< 2^64)
    moves(a, dst[2:], [None] * 6)
    a("s_branch %s" % lab_done)
    a.label(lab_uni)
    _uniform_limbs(a, dst, z, tt[0])
    a.label(lab_done)
    a("s_mov_b64 exec, %s" % sp(rest))
    a("s_cbranch_execnz %s" % lab_again)
    a("s_mov_b64 exec, %s" % sp(save))
    if wait:
        a("s_waitcnt vmcnt(0)")                      # boundary and pool loads
    a.cold()
    a.label(lab_slow)
    lane_class()
    a("s_branch %s" % lab_join)
    a.label(lab_loop)
    a("v_readfirstlane_b32 %s, %s" % (s(sc), v(cls)))
    a("v_cmp_eq_u32 vcc, %s, %s" % (s(sc), v(cls)))
    a("s_and_saveexec_b64 %s, vcc" % sp(rest))
    a("s_andn2_b64 %s, %s, exec" % (sp(rest), sp(rest)))   # lanes still to do
    a("s_branch %s" % lab_disp)
    # another group in this wave: its loads are in flight into other lanes
    # of dst; settle them before the next class writes dst
    a.label(lab_again)
    a("s_waitcnt vmcnt(0)")
    a("s_branch %s" % lab_loop)
    a.hot()


def h_leaf(a, bank, root, mask, dc=False, w32=False, ip=False):
    prologue(a, bank)
    if mask:
        load_masks(a, fld(bank, F_MOFF))
    lab_mem, lab_done = a.uniq("lmem"), a.uniq("ldone")
    if JIT:
        # compiled programs: the common case (generator mode, no leaf store,
        # aligned wave) behind one flag test, as in h_leafd
        def masked():
            if mask:
                a("s_waitcnt lgkmcnt(0)")
                for j in range(8):
                    a("v_and_b32 %s, %s, %s" % (v(X[j]), s(S_M + j), v(X[j])))
        lab_gen = a.uniq("lgen")
        a("s_bitcmp1_b32 %s, 0" % s(S_FAST))
        a("s_cbranch_scc0 %s" % lab_gen)
        _gen_leaf(a, bank, aligned=True)
        masked()
        a.label(lab_done)
        finish(a, bank, X, root, mask)
        a.cold()
        a.label(lab_gen)
        a("s_bitcmp1_b32 %s, 0" % IN["mode"])
        a("s_cbranch_scc0 %s" % lab_mem)
        _gen_leaf(a, bank, nested=True)
        masked()
        _store_soa(a, X, IN["lout"], fld(bank, F_C))
        a("s_branch %s" % lab_done)
        a.label(lab_mem)
        _soa_base(a, IN["leaves"], fld(bank, F_C))
        lane_offset(a, T[0])
        for j in range(8):
            a("global_load_dword %s, %s, %s" % (v(X[j]), v(T[0]), sp(S_T)))
            if j < 7:
                _soa_step(a)
        a("s_waitcnt vmcnt(0)")
        a("s_branch %s" % lab_done)
        a.hot()
        a.flush_cold()
        return
    a("s_bitcmp1_b32 %s, 0" % IN["mode"])
    a("s_cbranch_scc0 %s" % lab_mem)                 # (generator mode in line)
    _gen_leaf(a, bank)
    if mask:
        a("s_waitcnt lgkmcnt(0)")
        for j in range(8):
            a("v_and_b32 %s, %s, %s" % (v(X[j]), s(S_M + j), v(X[j])))
    _store_soa(a, X, IN["lout"], fld(bank, F_C), cold=True)
    a.label(lab_done)
    finish(a, bank, X, root, mask)
    a.cold()
    a.label(lab_mem)
    _soa_base(a, IN["leaves"], fld(bank, F_C))
    lane_offset(a, T[0])
    for j in range(8):
        a("global_load_dword %s, %s, %s" % (v(X[j]), v(T[0]), sp(S_T)))
        if j < 7:
            _soa_step(a)
    a("s_waitcnt vmcnt(0)")
    a("s_branch %s" % lab_done)
    a.hot()
    a.flush_cold()


def _wait_if_flagged(a: Asm, var: int):
    """LEAFD / RELOADD whose consumer is the very next record (the WAITD
    variant, chosen by the translator): the handler waits for its loads
    itself instead of a separate WAITVM record; static, no test."""
    if var & V_WAITD:
        a("s_waitcnt vmcnt(0)")


def h_leafd(a: Asm, bank: int, var: int):
    """256-bit LEAF into slot ``slot`` (the variant): the value is built
    straight in the slot's registers and its memory loads (input SoA, or the
    generator's boundary / pool lanes) are left in flight, so a run of leaves
    pays one memory latency at the WAITVM the translator puts before the
    first instruction that touches a pending slot."""
    slot = var & 15
    fd = [FB + 8 * slot + j for j in range(8)]
    prologue(a, bank)
    lab_mem, lab_done = a.uniq("lmem"), a.uniq("ldone")
    if JIT:
        # compiled programs: one flag test per leaf for the common case
        # (generator mode, no leaf store); the rest in a cold copy
        lab_gen = a.uniq("lgen")
        a("s_bitcmp1_b32 %s, 0" % s(S_FAST))
        a("s_cbranch_scc0 %s" % lab_gen)
        _gen_leaf(a, bank, dst=fd, wait=False, aligned=True)
        a.label(lab_done)
        _wait_if_flagged(a, var)
        dispatch(a, 1 - bank)
        a.cold()
        a.label(lab_gen)
        a("s_bitcmp1_b32 %s, 0" % IN["mode"])
        a("s_cbranch_scc0 %s" % lab_mem)
        _gen_leaf(a, bank, dst=fd, wait=False, nested=True)
        _store_soa(a, fd, IN["lout"], fld(bank, F_C), wait_vm=True)
        a("s_branch %s" % lab_done)
        a.label(lab_mem)
        _soa_base(a, IN["leaves"], fld(bank, F_C))
        lane_offset(a, T[0])
        for j in range(8):
            a("global_load_dword %s, %s, %s" % (v(fd[j]), v(T[0]), sp(S_T)))
            if j < 7:
                _soa_step(a)
        a("s_branch %s" % lab_done)
        a.hot()
        a.flush_cold()
        return
    a("s_bitcmp1_b32 %s, 0" % IN["mode"])
    a("s_cbranch_scc0 %s" % lab_mem)                 # (generator mode in line)
    _gen_leaf(a, bank, dst=fd, wait=False)
    _store_soa(a, fd, IN["lout"], fld(bank, F_C), wait_vm=True, cold=True)
    a.label(lab_done)
    _wait_if_flagged(a, var)
    dispatch(a, 1 - bank)
    a.cold()
    a.label(lab_mem)
    _soa_base(a, IN["leaves"], fld(bank, F_C))
    lane_offset(a, T[0])
    for j in range(8):
        a("global_load_dword %s, %s, %s" % (v(fd[j]), v(T[0]), sp(S_T)))
        if j < 7:
            _soa_step(a)
    a("s_branch %s" % lab_done)
    a.hot()
    a.flush_cold()


def h_reloadd(a: Asm, bank: int, var: int):
    """Scratch reload into slot ``slot`` (the variant) with the loads left in
    flight; the translator hoists it above earlier instructions that leave
    the slot and the spill slot alone, and puts a WAITVM before the first
    instruction that touches the slot."""
    fd = FB + 8 * (var & 15)
    prologue(a, bank)
    a("s_add_u32 %s, %s, %s" % (s(S_T), IN["scr"], s(fld(bank, F_IMM))))
    if var & V_NARROW:                 # one dword; limbs 1..7 of a one-limb value
        a("scratch_load_dword v%d, off, %s" % (fd, s(S_T)))
        moves(a, [fd + j for j in range(1, 8)], [None] * 7)
    else:
        a("scratch_load_dwordx4 v[%d:%d], off, %s" % (fd, fd + 3, s(S_T)))
        a("scratch_load_dwordx4 v[%d:%d], off, %s offset:16" % (fd + 4, fd + 7, s(S_T)))
    _wait_if_flagged(a, var)
    dispatch(a, 1 - bank)


def h_eqsel(a: Asm, bank: int, var: int):
    """One link of a lowered select-over-store chain, EQ fused with the ITE
    that consumes it (mg_api.cpp translate; the Bool is never stored):
      in place (default):  F[D] <- F[C]   where (F[A] == F[B]) != NEG
      GEN:                 F[D] <- (F[A] == F[B]) ? F[C] : F[IMM]
    The copies run under exec, two limbs per v_mov_b64."""
    prologue(a, bank)
    a.read_slot(Y, fld(bank, F_B))
    a.idx_on(fld(bank, F_A), "SRC0")
    for j in range(0, 8, 2):
        a("v_cmp_eq_u64_e64 %s, %s, %s" % (sp(S_T + j), vp(F[j]), vp(Y[j])))
    a.idx_off()
    a("s_and_b64 %s, %s, %s" % (sp(S_T), sp(S_T), sp(S_T + 2)))
    a("s_and_b64 %s, %s, %s" % (sp(S_T + 4), sp(S_T + 4), sp(S_T + 6)))
    a("s_and_b64 vcc, %s, %s" % (sp(S_T), sp(S_T + 4)))
    if var & V_GEN:
        a.read_slot(R, fld(bank, F_IMM))          # else value
        lab = exec_begin(a, None, S_T)
        a.read_slot(R, fld(bank, F_C))            # value taken, where equal
        exec_end(a, lab, S_T)
        a.write_slot(R, fld(bank, F_D))
    else:
        a.read_slot(Y, fld(bank, F_C))            # value taken
        lab = exec_begin(a, None, S_T, invert=bool(var & V_NEG))
        a.idx_on(fld(bank, F_D), "DST")
        moves(a, F, Y)
        a.idx_off()
        exec_end(a, lab, S_T)
    dispatch(a, 1 - bank)


# ---- the calldata word (ir.py _calldata_word) ---------------------------------

def h_bcast(a, bank, root, mask, dc=False, w32=False, ip=False):
    """F[D] = byte 0 of F[A] in all 32 bytes (the table's else byte, an
    8-bit value): one multiply by 0x01010101, four pair moves."""
    prologue(a, bank)
    a("s_mov_b32 %s, 0x1010101" % s(S_T))
    a.idx_on(fld(bank, F_A), "SRC0")
    a("v_mul_lo_u32 %s, %s, %s" % (v(R[0]), v(F[0]), s(S_T)))
    a.idx_off()
    a("v_mov_b32 %s, %s" % (v(R[1]), v(R[0])))
    a.idx_on(fld(bank, F_D), "DST")
    for j in range(0, 8, 2):
        a("v_mov_b64 %s, %s" % (vp(F[j]), vp(R[0])))
    a.idx_off()
    dispatch(a, 1 - bank)


def h_cdwe(a, bank, root, mask, dc=False, w32=False, ip=False):
    """One table entry of a calldata word: F[D] = F[A] with byte 31 - d set to
    F[C] & 0xff in the lanes where d = F[B] (= key - off) is below 32.  A
    wave with no such lane only copies (in place: nothing at all).  The
    byte's limb q = (31 - d) >> 2 is selected per limb by a compare (X[j]:
    the byte mask where q == j, else 0), then one v_bfi per limb."""
    prologue(a, bank)
    a.idx_on(fld(bank, F_B), "SRC0,SRC1,SRC2")
    a("v_or3_b32 %s, %s, %s, %s" % (v(T[1]), v(F[1]), v(F[2]), v(F[3])))
    a("v_or3_b32 %s, %s, %s, %s" % (v(T[2]), v(F[4]), v(F[5]), v(F[6])))
    a("s_set_gpr_idx_mode gpr_idx(SRC0)")
    a("v_or3_b32 %s, %s, %s, %s" % (v(T[1]), v(F[7]), v(T[1]), v(T[2])))
    a("v_mov_b32 %s, %s" % (v(T[0]), v(F[0])))
    a.idx_off()
    a("v_cmp_eq_u32_e64 %s, 0, %s" % (sp(S_T), v(T[1])))
    a("v_cmp_gt_u32 vcc, 32, %s" % v(T[0]))
    a("s_and_b64 vcc, vcc, %s" % sp(S_T))            # lanes whose key is a byte of the word
    if not ip:
        a.read_slot(R, fld(bank, F_A))
    done = a.uniq("cdwe")
    a("s_cbranch_vccz %s" % done)
    a("v_sub_u32 %s, 31, %s" % (v(T[2]), v(T[0])))               # byte position p
    a("v_lshrrev_b32 %s, 2, %s" % (v(T[3]), v(T[2])))            # its limb
    a("v_lshlrev_b32 %s, 3, %s" % (v(T[4]), v(T[2])))
    a("v_and_b32 %s, 24, %s" % (v(T[4]), v(T[4])))               # its shift in the limb
    a.idx_on(fld(bank, F_C), "SRC1")
    a("v_lshlrev_b32 %s, %s, %s" % (v(T[5]), v(T[4]), v(F[0])))  # value byte in place
    a.idx_off()
    a("v_mov_b32 %s, 0xff" % v(T[6]))
    a("v_lshlrev_b32 %s, %s, %s" % (v(T[6]), v(T[4]), v(T[6])))  # byte mask
    a("v_cndmask_b32_e64 %s, 0, %s, vcc" % (v(T[6]), v(T[6])))    # no hit: no byte
    for j in range(8):
        a("v_cmp_eq_u32_e64 %s, %d, %s" % (sp(S_T), j, v(T[3])))
        a("v_cndmask_b32_e64 %s, 0, %s, %s" % (v(X[j]), v(T[6]), sp(S_T)))
    if ip:
        a.idx_on(fld(bank, F_D), "SRC2,DST")
        for j in range(8):
            a("v_bfi_b32 %s, %s, %s, %s" % (v(F[j]), v(X[j]), v(T[5]), v(F[j])))
        a.idx_off()
    else:
        for j in range(8):
            a("v_bfi_b32 %s, %s, %s, %s" % (v(R[j]), v(X[j]), v(T[5]), v(R[j])))
    a.label(done)
    if not ip:
        a.write_slot(R, fld(bank, F_D))
    dispatch(a, 1 - bank)


def _prefix(a: Asm, out: int, n: int, pair: int):
    """v[out] = the low n bits set, n in 0..32 (32: all ones): the low half
    of (1 << n) - 1 from a 64-bit shift (a 32-bit shift by 32 is a shift by
    0); v[pair:pair+1] is scratch (even-aligned)."""
    a("v_lshlrev_b64 %s, %s, 1" % (vp(pair), v(n)))
    a("v_add_u32 %s, -1, %s" % (v(out), v(pair)))


def h_cdwx(a, bank, root, mask, dc=False, w32=False, ip=False):
    """The calldata word's size test: F[D] = F[A] with byte 31 - i cleared for
    every i < 32 where not (F[B] + i <s F[C]) (off, size; the add wraps at
    2^256).  With u = off ^ 2^255 and s' = size ^ 2^255 the test is the
    unsigned u + i < s'.  Without wrap (u <= 2^256 - 32) the valid bytes are
    the first n = (s' < u) ? 0 : min(s' - u, 32); lanes whose u + i wraps
    (off's top limb 0x7fffffff, then the exact test out of line) add the
    interval [K, min(32, K + s')) past the wrap point K = 2^256 - u.  The
    32-bit byte set is bit-reversed so nibble j covers limb j, and each
    nibble is spread to a byte mask (a 24-bit multiply puts bit k at bit
    8k, then t * 255)."""
    prologue(a, bank)
    a.read_slot(Y, fld(bank, F_B))                                 # off
    a.idx_on(fld(bank, F_C), "SRC0")                              # size - off, signed borrow
    a("v_sub_co_u32 %s, vcc, %s, %s" % (v(T[0]), v(F[0]), v(Y[0])))
    for j in range(1, 7):
        a("v_subb_co_u32 %s, vcc, %s, %s, vcc" % (v(T[j]), v(F[j]), v(Y[j])))
    a("s_set_gpr_idx_mode gpr_idx(SRC1)")
    a("v_xor_b32 %s, 0x80000000, %s" % (v(T[7]), v(F[7])))
    a.idx_off()
    a("v_xor_b32 %s, 0x80000000, %s" % (v(T[8]), v(Y[7])))
    a("v_subb_co_u32 %s, vcc, %s, %s, vcc" % (v(T[7]), v(T[7]), v(T[8])))
    a("s_mov_b64 %s, vcc" % sp(S_X))                             # size <s off
    a("v_or3_b32 %s, %s, %s, %s" % (v(T[1]), v(T[1]), v(T[2]), v(T[3])))
    a("v_or3_b32 %s, %s, %s, %s" % (v(T[1]), v(T[1]), v(T[4]), v(T[5])))
    a("v_or3_b32 %s, %s, %s, %s" % (v(T[1]), v(T[1]), v(T[6]), v(T[7])))
    a("v_min_u32 %s, 32, %s" % (v(T[0]), v(T[0])))
    a("v_cmp_ne_u32 vcc, 0, %s" % v(T[1]))
    a("v_cndmask_b32_e64 %s, %s, 32, vcc" % (v(T[0]), v(T[0])))
    a("v_cndmask_b32_e64 %s, %s, 0, %s" % (v(T[0]), v(T[0]), sp(S_X)))   # n
    wrap, done = a.uniq("cdxw"), a.uniq("cdxd")
    a("v_cmp_eq_u32 vcc, 0x7fffffff, %s" % v(Y[7]))
    a("s_cbranch_vccnz %s" % wrap)
    # no lane wraps: the valid bytes are the first n, so limb j keeps its
    # top min(max(n - 4(7 - j), 0), 4) bytes — with x_j = 8 * that, the
    # low word of (0xffffffff << 32) >> x_j (x_j <= 32: a 64-bit shift)
    a("v_cmp_gt_u32 vcc, 32, %s" % v(T[0]))                    # lanes missing a byte
    if not ip:
        a.read_slot(R, fld(bank, F_A))
    a("s_cbranch_vccz %s" % done)                              # every byte valid
    a("v_lshlrev_b32 %s, 3, %s" % (v(T[1]), v(T[0])))          # 8n
    a("s_mov_b32 %s, 0" % s(S_T))
    a("s_mov_b32 %s, -1" % s(S_T + 1))
    for j in range(8):
        k = 32 * (7 - j)
        if k:
            a("v_subrev_u32 %s, %d, %s" % (v(T[4]), k, v(T[1])))
            a("v_med3_i32 %s, %s, 0, 32" % (v(T[4]), v(T[4])))
        else:
            a("v_min_u32 %s, 32, %s" % (v(T[4]), v(T[1])))
        a("v_lshrrev_b64 %s, %s, %s" % (vp(T[2]), v(T[4]), sp(S_T)))
        if ip:
            a.idx_on(fld(bank, F_D), "SRC1,DST")
            a("v_and_b32 %s, %s, %s" % (v(F[j]), v(T[2]), v(F[j])))
            a.idx_off()
        else:
            a("v_and_b32 %s, %s, %s" % (v(R[j]), v(T[2]), v(R[j])))

    def spread_and():
        # T[2] = the 32-bit valid-byte set (bit i: byte 31 - i)
        a("v_cmp_ne_u32 vcc, -1, %s" % v(T[2]))
        if not ip:
            a.read_slot(R, fld(bank, F_A))
        a("s_cbranch_vccz %s" % done)                              # every byte valid
        a("v_bfrev_b32 %s, %s" % (v(T[2]), v(T[2])))               # bit 4j + k: limb j, byte k
        a("s_mov_b32 %s, 0x1010101" % s(S_T))
        for j in range(8):
            a("v_bfe_u32 %s, %s, %d, 4" % (v(T[3]), v(T[2]), 4 * j))
            a("v_mul_u32_u24 %s, 0x204081, %s" % (v(T[3]), v(T[3])))    # bit k -> bit 8k
            a("v_and_b32 %s, %s, %s" % (v(T[3]), s(S_T), v(T[3])))
            # x 255 (a 24-bit multiply would drop byte 3's bit): (t << 8) - t
            a("v_lshlrev_b32 %s, 8, %s" % (v(X[j]), v(T[3])))
            a("v_sub_u32 %s, %s, %s" % (v(X[j]), v(X[j]), v(T[3])))
        if ip:
            a.idx_on(fld(bank, F_D), "SRC1,DST")
            for j in range(8):
                a("v_and_b32 %s, %s, %s" % (v(F[j]), v(X[j]), v(F[j])))
            a.idx_off()
        else:
            for j in range(8):
                a("v_and_b32 %s, %s, %s" % (v(R[j]), v(X[j]), v(R[j])))
    a.label(done)
    if not ip:
        a.write_slot(R, fld(bank, F_D))
    dispatch(a, 1 - bank)
    a.cold()
    # some lane's off has the top limb 0x7fffffff: u + i may wrap at 2^256
    a.label(wrap)
    a("v_and_b32 %s, %s, %s" % (v(T[3]), v(Y[1]), v(Y[2])))
    for j in range(3, 7):
        a("v_and_b32 %s, %s, %s" % (v(T[3]), v(T[3]), v(Y[j])))
    a("v_cmp_eq_u32_e64 %s, -1, %s" % (sp(S_T), v(T[3])))
    a("s_and_b64 %s, %s, vcc" % (sp(S_T), sp(S_T)))                # u's upper limbs all ones
    a("v_sub_u32 %s, 0, %s" % (v(T[4]), v(Y[0])))                 # K = 2^32 - u_lo
    a("v_add_u32 %s, -1, %s" % (v(T[5]), v(T[4])))
    a("v_cmp_gt_u32 vcc, 31, %s" % v(T[5]))                        # K in 1..31
    a("s_and_b64 %s, %s, vcc" % (sp(S_T), sp(S_T)))
    a("v_cndmask_b32_e64 %s, 32, %s, %s" % (v(T[4]), v(T[4]), sp(S_T)))   # K (32: no wrap)
    a.idx_on(fld(bank, F_C), "SRC0,SRC1,SRC2")                    # min(s', 32)
    a("v_or3_b32 %s, %s, %s, %s" % (v(T[5]), v(F[1]), v(F[2]), v(F[3])))
    a("v_or3_b32 %s, %s, %s, %s" % (v(T[6]), v(F[4]), v(F[5]), v(F[6])))
    a("s_set_gpr_idx_mode gpr_idx(SRC1)")
    a("v_xor_b32 %s, 0x80000000, %s" % (v(T[7]), v(F[7])))
    a("v_min_u32 %s, 32, %s" % (v(T[8]), v(F[0])))
    a.idx_off()
    a("v_or3_b32 %s, %s, %s, %s" % (v(T[5]), v(T[5]), v(T[6]), v(T[7])))
    a("v_cmp_ne_u32 vcc, 0, %s" % v(T[5]))
    a("v_cndmask_b32_e64 %s, %s, 32, vcc" % (v(T[8]), v(T[8])))
    a("v_add_u32 %s, %s, %s" % (v(T[8]), v(T[4]), v(T[8])))
    a("v_min_u32 %s, 32, %s" % (v(T[8]), v(T[8])))                # end of the wrapped run
    a("v_min_u32 %s, %s, %s" % (v(T[0]), v(T[4]), v(T[0])))       # min(K, n)
    _prefix(a, T[2], T[0], T[2])
    _prefix(a, T[6], T[8], T[6])
    _prefix(a, T[8], T[4], T[8])
    a("v_bfi_b32 %s, %s, 0, %s" % (v(T[6]), v(T[8]), v(T[6])))    # [K, end)
    a("v_or_b32 %s, %s, %s" % (v(T[2]), v(T[2]), v(T[6])))
    spread_and()                                                   # not a prefix here
    a("s_branch %s" % done)
    a.hot()
    a.flush_cold()


def h_waitvm(a, bank, root, mask, dc=False, w32=False, ip=False):
    prologue(a, bank)
    a("s_waitcnt vmcnt(0)")
    dispatch(a, 1 - bank)


# ---------------------------------------------------------------------------
# heavy ops: per-(bank, variant) stubs copy the record to S_CUR and branch to
# a shared body; the body prefetches the next record into bank A
# ---------------------------------------------------------------------------

def far_jump(a: Asm, label: str):
    """Jump anywhere in the body (s_branch reaches only +-128 KiB): the
    target's offset from .Lbase is an assembler-resolved literal."""
    a("s_add_u32 %s, %s, (%s - .Lbase_%%=)" % (s(S_JMP), s(S_BASE), label))
    a("s_addc_u32 %s, %s, 0" % (s(S_JMP + 1), s(S_BASE + 1)))
    a("s_setpc_b64 %s" % sp(S_JMP))


def heavy_stub(a: Asm, bank: int, varbits: int, body: str):
    if JIT:
        a.lines.append("@@CALL %s %d" % (body, varbits))
        return
    b = BANK[bank]
    for k in range(0, 8, 2):
        a("s_mov_b64 %s, %s" % (sp(S_CUR + k), sp(b + k)))
    a("s_mov_b32 %s, %d" % (s(S_VAR), varbits))
    a("s_branch %s" % body)


def heavy_prologue(a: Asm):
    if not JIT:
        a("s_load_dwordx8 s[%d:%d], %s, %s" % (BANK[0], BANK[0] + 7, sp(S_CODE), s(S_IP)))
        a("s_add_u32 %s, %s, 32" % (s(S_IP), s(S_IP)))
    load_masks(a, cur(F_MOFF))     # MOFF always names a valid 8-word entry


def heavy_finish(a: Asm, res: List[int]):
    """Write (masked when variant bit1), fold ROOT when bit0, dispatch (A).
    The unmasked, non-root case runs straight through (no taken branch);
    the other two are out of line, placed after the dispatch."""
    lab_m, lab_wd, lab_r, lab_nr = a.uniq("hm"), a.uniq("hwd"), a.uniq("hr"), a.uniq("hnr")
    a("s_waitcnt lgkmcnt(0)")
    a("s_bitcmp1_b32 %s, 1" % s(S_VAR))
    a("s_cbranch_scc1 %s" % lab_m)
    a.write_slot(res, cur(F_D), None)
    a.label(lab_wd)
    a("s_bitcmp1_b32 %s, 0" % s(S_VAR))
    a("s_cbranch_scc1 %s" % lab_r)
    a.label(lab_nr)
    dispatch(a, 0)
    a.cold()
    a.label(lab_m)
    a.write_slot(res, cur(F_D), S_M)
    a("s_branch %s" % lab_wd)
    a.label(lab_r)
    a.root_and(v(res[0]))
    a("s_branch %s" % lab_nr)
    a.hot()
    a.flush_cold()


def col_product(a: Asm, x: List[int], y: List[int], ncols: int, out: Optional[List[int]] = None,
                hi_or: Optional[int] = None):
    """Product scanning of x*y over columns 0..ncols-1 with a 96-bit column
    accumulator: the aligned pair (A0:A1) takes every 64-bit product
    (v_mad_u64_u32), its carry-out goes to A2; the column digit is then A0
    and the accumulator shifts down one word.  Column c < 8 goes to out[c]
    (if given); with hi_or, columns >= 8 and the bits of columns < 8 outside
    the masks s[S_M+c] (loaded and waited for) are OR-ed into v[hi_or].
    Uses T4..T6 (T7 is read as the don't-care half of the shift's source
    pair), TMP, vcc, s[S_T+6:S_T+7]."""
    A0, A1, A2 = T[4], T[5], T[6]
    if hi_or is not None:
        a("v_mov_b32 %s, 0" % v(hi_or))
    for c in range(ncols):
        last = c == ncols - 1
        for n, i in enumerate(range(max(0, c - 7), min(c, 7) + 1)):
            j = c - i
            add = "0" if c == 0 else "v[%d:%d]" % (A0, A1)
            a("v_mad_u64_u32 v[%d:%d], %s, %s, %s, %s" % (
                A0, A1, sp(S_T + 6), v(x[i]), v(y[j]), add))
            if not last:
                # the column's first carry starts the overflow word afresh
                a("v_addc_co_u32_e64 %s, vcc, 0, %s, %s" % (v(A2), "0" if n == 0 else v(A2),
                                                            sp(S_T + 6)))
        if out is not None and c < 8:
            a("v_mov_b32 %s, %s" % (v(out[c]), v(A0)))
        if hi_or is not None:
            if c >= 8:
                a("v_or_b32 %s, %s, %s" % (v(hi_or), v(hi_or), v(A0)))
            else:
                a("v_bfi_b32 %s, %s, 0, %s" % (v(TMP), s(S_M + c), v(A0)))
                a("v_or_b32 %s, %s, %s" % (v(hi_or), v(hi_or), v(TMP)))
        if not last:                                  # (A0, A1) <- (A1, A2)
            a("v_pk_mov_b32 v[%d:%d], v[%d:%d], v[%d:%d] op_sel:[1,0]" % (A0, A1, A0, A1, A2, A2 + 1))


def low_product(a: Asm, x: List[int], y: List[int], out: List[int]):
    """out[0..7] = (x*y) mod 2^256 by product scanning, with the column
    accumulator placed so no digit needs a copy on even columns: column c
    even accumulates in the aligned pair (out[c], out[c+1]) (the digit stays
    in out[c]), column c odd in (A0, A1) with its digit copied to out[c]; one
    v_pk_mov_b32 per column moves (high word, carry word) on.  Column 0's
    single product cannot carry; the carries of column 6 would only reach
    column 8, so they are not tracked.  Uses T4..T6, vcc, s[S_T+6:S_T+7]."""
    A0, A1, A2 = T[4], T[5], T[6]
    for c in range(8):
        pair = (out[c], out[c + 1]) if c % 2 == 0 else (A0, A1)
        for n, i in enumerate(range(0, c + 1)):
            add = "0" if c == 0 else "v[%d:%d]" % pair
            a("v_mad_u64_u32 v[%d:%d], %s, %s, %s, %s" % (
                pair[0], pair[1], sp(S_T + 6), v(x[i]), v(y[c - i]), add))
            if 1 <= c <= 5:
                a("v_addc_co_u32_e64 %s, vcc, 0, %s, %s" % (v(A2), "0" if n == 0 else v(A2),
                                                            sp(S_T + 6)))
        if c % 2 == 1:
            a("v_mov_b32 %s, %s" % (v(out[c]), v(A0)))
            if c < 7:                                 # (out[c+1], out[c+2]) <- (A1, A2)
                a("v_pk_mov_b32 v[%d:%d], v[%d:%d], v[%d:%d] op_sel:[1,0]" % (
                    out[c + 1], out[c + 2], A0, A1, A2, A2 + 1))
        else:                                         # (A0, A1) <- (out[c+1], A2 | 0)
            a("v_pk_mov_b32 v[%d:%d], v[%d:%d], %s op_sel:[1,0]" % (
                A0, A1, out[c], out[c + 1], "0" if c == 0 else "v[%d:%d]" % (A2, A2 + 1)))


def h_mul(a, bank, root, mask, dc=False, w32=False, ip=False):
    """MUL in line in each (variant, bank) handler, unlike the other heavy
    ops: no record copy, no branch to a shared body, no run-time variant
    tests (the most frequent heavy op; ~100 instructions per copy)."""
    prologue(a, bank)
    if mask:
        load_masks(a, fld(bank, F_MOFF))
    a.read_slot(X, fld(bank, F_A))
    a.read_slot(Y, fld(bank, F_B))
    low_product(a, X, Y, R)
    finish(a, bank, R, root, mask)


def clz256(a: Asm, vals: List[int], out: int, t: List[int]):
    """Leading zeros of a 256-bit value (256 for zero): min over limbs of
    (7-j)*32 + ffbh(limb j), ffbh(0) = ~0 kept saturated by a clamped add.
    t: 8 temps (may include out).  Clobbers s[S_T..S_T+7]."""
    for j in range(8):
        a("s_movk_i32 %s, 0x%x" % (s(S_T + j), (7 - j) * 32))
    for j in range(8):
        a("v_ffbh_u32 %s, %s" % (v(t[j]), v(vals[j])))
        a("v_add_u32_e64 %s, %s, %s clamp" % (v(t[j]), v(t[j]), s(S_T + j)))
    a("v_min3_u32 %s, %s, %s, %s" % (v(t[0]), v(t[0]), v(t[1]), v(t[2])))
    a("v_min3_u32 %s, %s, %s, %s" % (v(t[3]), v(t[3]), v(t[4]), v(t[5])))
    a("v_min3_u32 %s, %s, %s, %s" % (v(out), v(t[0]), v(t[3]), v(t[6])))
    a("s_movk_i32 %s, 0x100" % s(S_T))
    a("v_min3_u32 %s, %s, %s, %s" % (v(out), v(out), v(t[7]), s(S_T)))


def body_umulno(a: Asm):
    """R0 = (x*y < 2^W).  With p, q the bit lengths of x and y,
    2^(p+q-2) <= x*y < 2^(p+q): no overflow when p + q <= W, overflow when
    p + q >= W + 2.  Only the lanes with p + q == W + 1 need the product;
    the 512-bit product (columns >= W OR-ed; the width masks are all-ones
    for W = 256) runs only when some lane of the wave has one."""
    a.label(".Lbody_UMULNO_%=")
    heavy_prologue(a)
    a.read_slot(X, cur(F_A))
    a.read_slot(Y, cur(F_B))
    lab = a.uniq("unf")
    # W = 256 and both operands >= 2^128 in every active lane (90 % of the
    # C2 corpus's UMULNO waves): p + q >= 258, every product overflows —
    # no bit lengths needed (round 5)
    lab_gen = a.uniq("ung")
    a("s_cmp_eq_u32 %s, 0x100" % s(cur(F_W)))
    a("s_cbranch_scc0 %s" % lab_gen)
    a("v_or3_b32 %s, %s, %s, %s" % (v(T[0]), v(X[4]), v(X[5]), v(X[6])))
    a("v_or_b32 %s, %s, %s" % (v(T[0]), v(T[0]), v(X[7])))
    a("v_or3_b32 %s, %s, %s, %s" % (v(T[1]), v(Y[4]), v(Y[5]), v(Y[6])))
    a("v_or_b32 %s, %s, %s" % (v(T[1]), v(T[1]), v(Y[7])))
    a("v_cmp_ne_u32_e64 %s, 0, %s" % (sp(S_X + 4), v(T[0])))
    a("v_cmp_ne_u32 vcc, 0, %s" % v(T[1]))
    a("s_and_b64 vcc, vcc, %s" % sp(S_X + 4))
    a("s_cmp_eq_u64 vcc, exec")
    a("s_cbranch_scc0 %s" % lab_gen)
    a("s_mov_b64 %s, 0" % sp(S_X + 4))                 # no lane is free of overflow
    a("s_branch %s" % lab)
    a.label(lab_gen)
    sz = T[8]                                   # clz(x) + clz(y) = 512 - (p + q)
    clz256(a, X, sz, [T[8], T[9], T[10], T[11], T[0], T[1], T[2], T[3]])
    clz256(a, Y, T[4], [T[4], T[5], T[6], T[7], T[0], T[1], T[2], T[3]])
    a("v_add_u32 %s, %s, %s" % (v(sz), v(sz), v(T[4])))
    a("s_sub_u32 %s, 511, %s" % (s(S_X), s(cur(F_W))))                  # 511 - W
    a("v_cmp_eq_u32_e64 %s, %s, %s" % (sp(S_X + 2), s(S_X), v(sz)))     # p + q == W + 1
    a("v_cmp_lt_u32_e64 %s, %s, %s" % (sp(S_X + 4), s(S_X), v(sz)))     # p + q <= W
    a("s_cmp_eq_u64 %s, 0" % sp(S_X + 2))
    a("s_cbranch_scc1 %s" % lab)
    a("s_waitcnt lgkmcnt(0)")                   # the width masks
    col_product(a, X, Y, 16, hi_or=T[7])
    a("v_cmp_eq_u32 vcc, 0, %s" % v(T[7]))
    a("s_and_b64 vcc, vcc, %s" % sp(S_X + 2))
    a("s_or_b64 %s, %s, vcc" % (sp(S_X + 4), sp(S_X + 4)))
    a.label(lab)
    a("v_cndmask_b32_e64 %s, 0, 1, %s" % (v(R[0]), sp(S_X + 4)))
    a("v_mov_b32 %s, 0" % v(R[1]))
    for j in range(2, 8, 2):
        a("v_mov_b64 %s, 0" % vp(R[j]))
    a("s_and_b32 %s, %s, 1" % (s(S_VAR), s(S_VAR)))      # Bool result: never masked
    heavy_finish(a, R)


# ---- per-lane shifts ------------------------------------------------------

def exec_begin(a: Asm, mask: Optional[int], save: int, invert: bool = False,
               skip: bool = False) -> str:
    """Narrow exec to the lanes of s[mask:mask+1] (vcc if None; or the
    complement); returns the label that exec_end places.  VALU under a
    narrowed exec writes only those lanes, so a conditional update costs one
    plain instruction instead of a compute + v_cndmask pair.  The blocks are
    short, so by default there is no branch over an empty one: a taken
    branch (an instruction-fetch redirect) costs more than a few
    instructions issued with exec = 0 (+1.5 % corpus, profiles/r02/
    ab_noskip.log); ``skip`` adds it.  Clobbers s[save:save+1] and scc."""
    lab = a.uniq("xm")
    # one instruction saves exec and narrows it (andn1: exec &= ~mask)
    a("s_%s_saveexec_b64 %s, %s" % ("andn1" if invert else "and", sp(save),
                                    "vcc" if mask is None else sp(mask)))
    if skip:
        a("s_cbranch_execz %s" % lab)
    return lab


def exec_end(a: Asm, lab: str, save: int):
    a.label(lab)
    a("s_mov_b64 exec, %s" % sp(save))


def moves(a: Asm, dsts: List[int], srcs: List[Optional[int]]):
    """dsts[i] <- srcs[i] (None = 0) in list order, two limbs per instruction
    where the destinations form an even-aligned pair: v_mov_b64 when the
    sources do too, else v_pk_mov_b32 picking each half from its aligned
    source pair (full rate, profiles/r01/ubench2.log).  The caller orders
    the list so no source is overwritten before it is read (a pair reads
    both sources before writing)."""
    i = 0
    while i < len(dsts):
        if i + 1 < len(dsts) and abs(dsts[i + 1] - dsts[i]) == 1 and min(dsts[i], dsts[i + 1]) % 2 == 0:
            lo, hi = (i, i + 1) if dsts[i + 1] == dsts[i] + 1 else (i + 1, i)
            dl, sl, sh = dsts[lo], srcs[lo], srcs[hi]
            if sl is None and sh is None:
                a("v_mov_b64 %s, 0" % vp(dl))
            elif sl is not None and sh == sl + 1 and sl % 2 == 0:
                a("v_mov_b64 %s, %s" % (vp(dl), vp(sl)))
            else:
                o0 = "0" if sl is None else vp(sl & ~1)
                o1 = "0" if sh is None else vp(sh & ~1)
                a("v_pk_mov_b32 %s, %s, %s op_sel:[%d,%d]" % (
                    vp(dl), o0, o1, 0 if sl is None else sl & 1, 0 if sh is None else sh & 1))
            i += 2
            continue
        a("v_mov_b32 %s, %s" % (v(dsts[i]), "0" if srcs[i] is None else v(srcs[i])))
        i += 1


def _barrel(a: Asm, t: List[int], q: int, nl: int, left: bool, save: int,
            live: Optional[int] = None, fill: Optional[int] = None):
    hi = nl if live is None else live
    for st in (1, 2, 4):
        a("v_and_b32 %s, %d, %s" % (v(TMP), st, v(q)))
        a("v_cmp_ne_u32 vcc, 0, %s" % v(TMP))
        lab = exec_begin(a, None, save)
        if left:
            top = min(nl, hi + st)
            js = list(reversed(range(top)))
            moves(a, [t[j] for j in js], [t[j - st] if j - st >= 0 else None for j in js])
            hi = top
        else:
            moves(a, [t[j] for j in range(nl)], [t[j + st] if j + st < nl else fill
                                                 for j in range(nl)])
        exec_end(a, lab, save)


def barrel_right(a: Asm, t: List[int], q: int, nl: int, save: int, fill: Optional[int] = None):
    """t[0..nl-1] = t >> (32*q) limbs (q per lane in v[q] < 8), filled with
    zeros or with v[fill] (the sign word of an arithmetic shift); each stage
    moves only the lanes that take it (under exec)."""
    _barrel(a, t, q, nl, False, save, fill=fill)


def barrel_left(a: Asm, t: List[int], q: int, nl: int, save: int, live: Optional[int] = None):
    """t[0..nl-1] = t << (32*q) limbs (q < 8), zero fill; ``live`` = number
    of possibly-nonzero low limbs on entry (known-zero moves are skipped)."""
    _barrel(a, t, q, nl, True, save, live)


def bitshift_right(a: Asm, t: List[int], b: int, n_out: int):
    """t[j] = (t[j+1]:t[j]) >> b for j < n_out (t[n_out] must exist)."""
    for j in range(n_out):
        a("v_alignbit_b32 %s, %s, %s, %s" % (v(t[j]), v(t[j + 1]), v(t[j]), v(b)))


def bitshift_left(a: Asm, t: List[int], c: int, bz: int, nl: int, save: int):
    """t[j] = t[j] << b | t[j-1] >> (32-b), j = nl-1..0 (t[-1] = 0), for the
    lanes with b != 0 (c = 32 - b; s[bz:bz+1] = lanes with b == 0, which keep
    t unchanged: v_alignbit cannot shift by 32)."""
    lab = exec_begin(a, bz, save, invert=True)
    for j in reversed(range(nl)):
        lo = v(t[j - 1]) if j > 0 else "0"
        a("v_alignbit_b32 %s, %s, %s, %s" % (v(t[j]), v(t[j]), lo, v(c)))
    exec_end(a, lab, save)


def h_shift(kind: str):
    """SHL / LSHR / ASHR of F[a] by F[b] at width W, in line in each
    (variant, bank) handler (like MUL: no shared body, static variant)."""
    def h(a, bank, root, mask, dc=False, w32=False, ip=False):
        prologue(a, bank)
        if mask:
            load_masks(a, fld(bank, F_MOFF))
        shift_core(a, kind, fld(bank, F_A), fld(bank, F_B), fld(bank, F_W), mask)
        finish(a, bank, X, root, mask and kind != "LSHR")   # LSHR: canonical
    return h


def shift_core(a: Asm, kind: str, fa: int, fb: int, fw: int, masked: bool):
    """X = F[fa] shifted by F[fb] at the width in s[fw]; ASHR sign-extends
    from that width first when ``masked`` (the masks S_M are loading)."""
    a.read_slot(X, fa)
    over = S_X                     # s[88:89] lanes shifting by >= W
    # the shift amount is used straight from the file (all three sources of
    # the or3 indexed: limbs 1..6 of F[b]), no staging copy
    a.idx_on(fb, "SRC0,SRC1,SRC2")
    a("v_or3_b32 %s, %s, %s, %s" % (v(T[0]), v(F[1]), v(F[2]), v(F[3])))
    a("v_or3_b32 %s, %s, %s, %s" % (v(T[1]), v(F[4]), v(F[5]), v(F[6])))
    a("s_set_gpr_idx_mode gpr_idx(SRC0)")
    a("v_or3_b32 %s, %s, %s, %s" % (v(T[0]), v(F[7]), v(T[0]), v(T[1])))
    a("v_cmp_ge_u32_e64 %s, %s, %s" % (sp(S_T), v(F[0]), s(fw)))
    a("v_bfe_u32 %s, %s, 5, 3" % (v(T[2]), v(F[0])))         # q (over lanes masked later)
    a("v_and_b32_e64 %s, %s, 31" % (v(T[3]), v(F[0])))      # b
    a.idx_off()
    a("v_cmp_ne_u32_e64 %s, 0, %s" % (sp(over), v(T[0])))
    a("s_or_b64 %s, %s, %s" % (sp(over), sp(over), sp(S_T)))
    fill = None
    if kind == "ASHR":
        if masked:
            a("s_waitcnt lgkmcnt(0)")
            sext(a, X, fw, S_M, T[4], S_T)
        a("v_ashrrev_i32 %s, 31, %s" % (v(T[4]), v(X[7])))   # the sign word
        fill = T[4]
    lab_all = a.uniq("sho")
    a("s_andn2_b64 %s, exec, %s" % (sp(S_T), sp(over)))
    a("s_cbranch_scc0 %s" % lab_all)                 # every lane shifts by >= W
    if kind == "SHL":
        a("v_sub_u32 %s, 32, %s" % (v(T[5]), v(T[3])))
        a("v_cmp_eq_u32_e64 %s, 0, %s" % (sp(S_X + 2), v(T[3])))
        barrel_left(a, X, T[2], 8, S_T)
        bitshift_left(a, X, T[5], S_X + 2, 8, S_T)
    else:                          # ASHR fills with the sign word directly
        a("v_mov_b32 %s, %s" % (v(R[0]), "0" if fill is None else v(fill)))
        t = X + [R[0]]
        barrel_right(a, t, T[2], 8, S_T, fill)
        bitshift_right(a, t, T[3], 8)
    a.label(lab_all)
    if fill is not None:
        a("v_mov_b32 %s, %s" % (v(T[5]), v(fill)))
    lab = exec_begin(a, over, S_T)                   # shift >= W: 0 or sign fill
    moves(a, X, [None if fill is None else T[4 + (j & 1)] for j in range(8)])
    exec_end(a, lab, S_T)


# ---- division ---------------------------------------------------------------
#
# Unsigned 256/256 Knuth D on 32-bit digits: normalise by sh = clz(v) (limbs
# + bits) so vn's top digit is vn[7]; un = u << sh (17 digits); quotient
# digit j (7..0) from un[j+8], un[j+7] with the Moller-Granlund reciprocal of
# d = vn[7] (two corrections give the exact 2-by-1 quotient, at most two above
# the true digit); multiply-subtract; add back (at most twice) where negative.
# An iteration is skipped when no lane of the wave has un[j+8] != 0 or
# un[j+7] >= d (its quotient digit is then 0 and nothing changes).
# Registers: u = X, v = Y on entry; un = X ++ R ++ [T0]; vn = Y;
# b/c = T2/T3 (b kept for the remainder); digit temps T4..T11.

# Division's wave-uniform exits and paths (rounds 3-5; each was an A/B knob,
# retired in round 6 with its losing side): the dividend is shifted by bits
# before limbs; limb-barrel stages of DIV_STAGE_SKIP or more limbs branch over
# an empty lane mask; a wave whose divisors all keep their top limb jumps to
# quotient digit 0 and computes the reciprocal only if some lane needs that
# digit; the one-limb short division's second correction sits behind a
# branch; waves whose divisors all fit 64 bits take Moller-Granlund 3-by-2
# steps; a wave dividing by zero everywhere skips the division.
DIV_M = {4: 48, 2: 50, 1: 52}   # limb-shift stage masks (bank B: free in heavy bodies)
DIV_Z6 = 54                     # lanes with vn[0..5] == 0 (bank B)
DIV_STAGE_SKIP = 6
DIV_Z4 = S_CUR + F_C            # lanes with vn[0..3] == 0 (record fields c, imm:
                                # unused by division)


def _stage(a: Asm, t: List[int], st: int, nl: int, left: bool, mask: int,
           live: Optional[int] = None) -> int:
    """One limb-barrel stage: shift t by st limbs in the lanes of s[mask]
    (under exec; zero fill).  Returns the new number of live low limbs.
    Stages of at least DIV_STAGE_SKIP limbs branch over an empty mask (a
    wave of full-width divisors — every uniform-class divisor leaf under
    generator v8 — needs none of them)."""
    n = min(nl, (nl if live is None else live) + st) if left else nl
    lab = exec_begin(a, mask, S_T + 2, skip=n >= DIV_STAGE_SKIP)
    if left:
        hi = nl if live is None else live
        top = min(nl, hi + st)
        js = list(reversed(range(top)))
        moves(a, [t[j] for j in js], [t[j - st] if j - st >= 0 else None for j in js])
    else:
        top = nl
        moves(a, [t[j] for j in range(nl)], [t[j + st] if j + st < nl else None for j in range(nl)])
    exec_end(a, lab, S_T + 2)
    return top


def udivrem(a: Asm, want_rem: bool, z: int):
    """X / Y: quotient -> R; remainder (want_rem) -> X; s[z:z+1] <- lanes
    with Y == 0, which compute 0 / 1 instead (quotient and remainder 0; the
    caller applies SMT-LIB's x/0 rules).  Normalisation shifts Y left until its top limb is nonzero,
    4, 2 then 1 limbs at a time in the lanes whose top limbs are zero (the
    stage masks stay in s[48:53] for the dividend and the remainder), then
    by b = clz(top limb) bits.  Registers: un = X ++ R ++ [T0]; vn = Y;
    b/c = T2/T3 (b kept for the remainder); pairs T4:T5, T6:T7, T8:T9
    (64-bit tuples start even on gfx950); dinv = T10.  Clobbers Y, T, vcc,
    s[S_T..S_T+7], s[48:53]."""
    un = X + R + [T[0]]
    vn = Y
    b, c, dinv = T[2], T[3], T[10]
    bz = S_T + 4
    # every active lane's divisor fits two limbs: out of line, where one limb
    # (the one-limb short division) or two (3-by-2 steps) is decided
    lab_done = a.uniq("dsd")
    t = T[4]
    lab_fit64, lab_two = a.uniq("d64"), a.uniq("d2l")
    a("v_or3_b32 %s, %s, %s, %s" % (v(t), v(Y[2]), v(Y[3]), v(Y[4])))
    a("v_or3_b32 %s, %s, %s, %s" % (v(t), v(t), v(Y[5]), v(Y[6])))
    a("v_or_b32 %s, %s, %s" % (v(t), v(t), v(Y[7])))
    a("v_cmp_eq_u32 vcc, 0, %s" % v(t))
    a("s_cmp_eq_u64 vcc, exec")
    a("s_cbranch_scc1 %s" % lab_fit64)
    a.cold()
    a.label(lab_fit64)
    a("v_cmp_eq_u32 vcc, 0, %s" % v(Y[1]))
    a("s_cmp_eq_u64 vcc, exec")
    a("s_cbranch_scc0 %s" % lab_two)
    # every active lane divides by zero (11 % of the C2 corpus's
    # division waves): quotient and remainder 0 as the contract says,
    # the caller applies SMT-LIB's x/0 rules
    lab_zero = a.uniq("dz")
    a("v_cmp_eq_u32_e64 %s, 0, %s" % (sp(z), v(Y[0])))
    a("s_cmp_eq_u64 %s, exec" % sp(z))
    a("s_cbranch_scc1 %s" % lab_zero)
    _udivrem_short(a, want_rem, z)
    a("s_branch %s" % lab_done)
    a.label(lab_zero)
    moves(a, (X if want_rem else []) + R, [None] * (16 if want_rem else 8))
    a("s_branch %s" % lab_done)
    a.label(lab_two)
    _udivrem_short2(a, want_rem, z)
    a("s_branch %s" % lab_done)
    a.hot()
    for j in range(0, 8, 2):
        a("v_mov_b64 %s, 0" % vp(R[j]))
    a("v_mov_b32 %s, 0" % v(T[0]))                                       # un[16]
    a("v_cmp_eq_u64_e64 %s, 0, %s" % (sp(DIV_M[4]), vp(Y[4])))
    a("v_cmp_eq_u64_e64 %s, 0, %s" % (sp(S_T), vp(Y[6])))
    a("s_and_b64 %s, %s, %s" % (sp(DIV_M[4]), sp(DIV_M[4]), sp(S_T)))
    _stage(a, vn, 4, 8, True, DIV_M[4])
    a("v_cmp_eq_u64_e64 %s, 0, %s" % (sp(DIV_M[2]), vp(Y[6])))
    _stage(a, vn, 2, 8, True, DIV_M[2])
    a("v_cmp_eq_u32_e64 %s, 0, %s" % (sp(DIV_M[1]), v(Y[7])))
    _stage(a, vn, 1, 8, True, DIV_M[1])
    a("v_cmp_eq_u32_e64 %s, 0, %s" % (sp(z), v(Y[7])))                  # Y == 0
    a("v_ffbh_u32 %s, %s" % (v(b), v(Y[7])))
    a("v_min_u32 %s, 31, %s" % (v(b), v(b)))                            # Y == 0: 1 << 255
    a("v_cndmask_b32_e64 %s, %s, 1, %s" % (v(Y[7]), v(Y[7]), sp(z)))
    a("v_sub_u32 %s, 32, %s" % (v(c), v(b)))
    a("v_cmp_eq_u32_e64 %s, 0, %s" % (sp(bz), v(b)))
    bitshift_left(a, vn, c, bz, 8, S_T)
    # lanes dividing by zero divide 0 instead (quotient and remainder 0; the
    # caller gives them their SMT-LIB result), so they never keep a quotient
    # digit of the wave alive (a divisor of 1 would need all eight)
    lab = exec_begin(a, z, S_T)
    moves(a, X, [None] * 8)
    exec_end(a, lab, S_T)
    # the dividend's bits first (9 limbs: u << b, the top limb un[8] = 0 on
    # entry), then its limbs: 9 funnels instead of 17 after the barrel
    bitshift_left(a, un, c, bz, 9, S_T)
    live = 9
    for st in (4, 2, 1):
        live = _stage(a, un, st, 17, True, DIV_M[st], live)
    # lanes whose normalised divisor has its low 4 / 6 digits zero: a
    # quotient digit's multiply-subtract starts at digit 4 / 6 when every
    # lane with a nonzero digit is one of them (qh * 0 changes nothing)
    t = T[4]
    a("v_or3_b32 %s, %s, %s, %s" % (v(t), v(vn[0]), v(vn[1]), v(vn[2])))
    a("v_or_b32 %s, %s, %s" % (v(t), v(t), v(vn[3])))
    a("v_cmp_eq_u32_e64 %s, 0, %s" % (sp(DIV_Z4), v(t)))
    a("v_or3_b32 %s, %s, %s, %s" % (v(t), v(t), v(vn[4]), v(vn[5])))
    a("v_cmp_eq_u32_e64 %s, 0, %s" % (sp(DIV_Z6), v(t)))
    d = vn[7]
    # a lane whose divisor moved q limbs has un[k] = 0 for k >= 9 + q and
    # un[8 + q] < 2^b <= d, so its quotient digits j > q are zero and their
    # tests below skip; when no lane moved its divisor (a wave of full-width
    # divisors; zero divisors excluded, they divide 0) only digit 0 can be
    # nonzero: one scalar test instead of seven per-digit VALU tests (round 5),
    # taken before the reciprocal, which such a wave then computes only when
    # some lane needs digit 0
    lab_j0, lab_rem = a.uniq("dj0"), a.uniq("drm")
    a("s_or_b64 %s, %s, %s" % (sp(S_T), sp(DIV_M[4]), sp(DIV_M[2])))
    a("s_or_b64 %s, %s, %s" % (sp(S_T), sp(S_T), sp(DIV_M[1])))
    a("s_andn2_b64 %s, %s, %s" % (sp(S_T), sp(S_T), sp(z)))
    a("s_cbranch_scc0 %s" % lab_j0)
    _reciprocal(a, d, dinv)
    a("v_mov_b32 %s, 0" % v(T[9]))                                  # RH of the digit loop

    def digit_test(j, skip):
        a("v_cmp_ne_u32_e64 %s, 0, %s" % (sp(S_T), v(un[j + 8])))
        a("v_cmp_ge_u32_e64 %s, %s, %s" % (sp(S_T + 2), v(un[j + 7]), v(d)))
        a("s_or_b64 vcc, %s, %s" % (sp(S_T), sp(S_T + 2)))
        a("s_cbranch_vccz %s" % skip)

    for j in reversed(range(8)):
        skip = a.uniq("dvs")
        digit_test(j, skip)
        _div_digit(a, un, vn, j, d, dinv)
        a.label(skip)
    a("s_branch %s" % lab_rem)
    a.label(lab_j0)
    digit_test(0, lab_rem)
    _reciprocal(a, d, dinv)
    a("v_mov_b32 %s, 0" % v(T[9]))
    _div_digit(a, un, vn, 0, d, dinv)
    a.label(lab_rem)
    if want_rem:
        # remainder = un[0..8] >> sh; un[8] now holds a quotient digit: use 0
        a("v_mov_b32 %s, 0" % v(T[0]))
        t = X + [T[0]]
        for st in (1, 2, 4):
            _stage(a, t, st, 9, False, DIV_M[st])
        bitshift_right(a, t, b, 8)
    a.label(lab_done)


def _udivrem_short(a: Asm, want_rem: bool, z: int):
    """udivrem when every active lane's divisor Y fits 32 bits (wave-uniform:
    no limb barrel, no multiply-subtract): d = Y[0] << b normalised, u =
    X << b over 9 limbs, then eight 2-by-1 steps with the reciprocal
    (r:u[j]) / d -> quotient digit R[j], remainder r (r < d throughout),
    remainder = r >> b.  Same contract as udivrem: lanes with Y == 0 divide
    0 by 1 (s[z:z+1] marks them).  Registers: d = Y0, b = T2, c / r = T3,
    A = T4:T5, P = T6:T7, CR = T8, dinv = T10, QH = T11."""
    d, b, c, dinv = Y[0], T[2], T[3], T[10]
    A0, A1, Q0, Q1, CR, t, QH = T[4], T[5], T[6], T[7], T[8], T[9], T[11]
    r = A1                        # the running remainder, hi half of the mad addend
    bz = S_T + 4
    a("v_cmp_eq_u32_e64 %s, 0, %s" % (sp(z), v(d)))                   # Y == 0
    a("v_cndmask_b32_e64 %s, %s, 1, %s" % (v(d), v(d), sp(z)))
    lab = exec_begin(a, z, S_T)
    moves(a, X, [None] * 8)
    exec_end(a, lab, S_T)
    a("v_ffbh_u32 %s, %s" % (v(b), v(d)))                              # d >= 1: 0..31
    a("v_lshlrev_b32 %s, %s, %s" % (v(d), v(b), v(d)))
    a("v_sub_u32 %s, 32, %s" % (v(c), v(b)))
    a("v_cmp_eq_u32_e64 %s, 0, %s" % (sp(bz), v(b)))
    a("v_mov_b32 %s, 0" % v(R[0]))
    bitshift_left(a, X + [R[0]], c, bz, 9, S_T)                       # u = X << b
    _reciprocal(a, d, dinv)
    a("v_mov_b32 %s, %s" % (v(r), v(R[0])))                           # r = u[8] < d
    lt = sp(S_T + 2)
    for j in reversed(range(8)):
        # Moller-Granlund 2-by-1 (their Algorithm 4): (Q1:Q0) = dinv * r +
        # (r:u[j]); q = Q1 + 1; r' = u[j] - q * d; r' > Q0: q--, r' += d.  The
        # second correction (r' >= d: q++, r' -= d) is the paper's "unlikely"
        # one: a branch over it (round 5: 14 -> 10 VALU per digit; the
        # remainder stays in the addend's high half, r = A1)
        a("v_mov_b32 %s, %s" % (v(A0), v(X[j])))
        a("v_mad_u64_u32 v[%d:%d], %s, %s, %s, v[%d:%d]" % (Q0, Q1, sp(S_T + 6), v(dinv), v(r),
                                                           A0, A1))
        a("v_add_u32 %s, 1, %s" % (v(QH), v(Q1)))
        a("v_mul_lo_u32 %s, %s, %s" % (v(t), v(QH), v(d)))
        a("v_sub_u32 %s, %s, %s" % (v(CR), v(A0), v(t)))
        a("v_cmp_gt_u32_e64 %s, %s, %s" % (lt, v(CR), v(Q0)))           # r' > q0: q--, r' += d
        a("v_subb_co_u32_e64 %s, %s, %s, 0, %s" % (v(R[j]), sp(S_T + 4), v(QH), lt))
        a("v_cndmask_b32_e64 %s, 0, %s, %s" % (v(t), v(d), lt))
        a("v_add_u32 %s, %s, %s" % (v(r), v(CR), v(t)))
        a("v_cmp_ge_u32 vcc, %s, %s" % (v(r), v(d)))                     # r' >= d: q++, r' -= d
        skip = a.uniq("dss")
        a("s_cbranch_vccz %s" % skip)
        lab = exec_begin(a, None, S_T + 2)
        a("v_add_u32 %s, 1, %s" % (v(R[j]), v(R[j])))
        a("v_sub_u32 %s, %s, %s" % (v(r), v(r), v(d)))
        exec_end(a, lab, S_T + 2)
        a.label(skip)
    if want_rem:
        a("v_lshrrev_b32 %s, %s, %s" % (v(X[0]), v(b), v(r)))
        moves(a, X[1:], [None] * 7)


def _udivrem_short2(a: Asm, want_rem: bool, z: int):
    """udivrem when every active lane's divisor Y fits 64 bits (wave-uniform;
    some lane needs the second limb): the divisor is normalised to a 64-bit
    d = d1:d0 with its top bit set (lanes below 2^32 move up one limb, with
    the dividend), u = X << that shift over 10 limbs, then eight Moller-
    Granlund 3-by-2 steps (their Algorithm 5, with the 3/2 reciprocal of
    Algorithm 6) bring in one dividend limb each: (r1:r0:u[j]) / d ->
    quotient digit R[j], remainder r1:r0 < d.  No limb barrel, no multiply-
    subtract chain, no per-digit tests.  Same contract as udivrem (lanes
    with Y == 0 divide 0 by 1, s[z:z+1] marks them).  Registers: d0 / d1 =
    Y0 / Y1, b = T2, p = T3, r = T4:T5 (r0 low), Q = T6:T7, P = T8:T9,
    dinv = T10; s[52:53] = lanes shifted by a limb."""
    d0, d1 = Y[0], Y[1]
    b, p, dinv = T[2], T[3], T[10]
    r0, r1, q0, q1, t0, t1 = T[4], T[5], T[6], T[7], T[8], T[9]
    lq = DIV_M[1]
    un = X + [R[0], R[1]]
    dd = vp(Y[0])                                   # (d1:d0) as one 64-bit operand
    a("v_or_b32 %s, %s, %s" % (v(r0), v(d0), v(d1)))
    a("v_cmp_eq_u32_e64 %s, 0, %s" % (sp(z), v(r0)))                   # Y == 0
    a("v_cndmask_b32_e64 %s, %s, 1, %s" % (v(d0), v(d0), sp(z)))
    lab = exec_begin(a, z, S_T)
    moves(a, X, [None] * 8)
    exec_end(a, lab, S_T)
    a("v_mov_b64 %s, 0" % vp(R[0]))                                   # un[8], un[9]
    # divisors below 2^32 (d1 == 0) move up one limb, the dividend with them
    a("v_cmp_eq_u32_e64 %s, 0, %s" % (sp(lq), v(d1)))
    lab = exec_begin(a, lq, S_T)
    moves(a, [d1, d0], [d0, None])
    moves(a, [R[0]] + [X[j] for j in reversed(range(8))],
          [X[7]] + [X[j - 1] if j else None for j in reversed(range(8))])
    exec_end(a, lab, S_T)
    # then by b = clz(d1) bits (d1 != 0 in every lane now)
    bz = S_T + 4
    a("v_ffbh_u32 %s, %s" % (v(b), v(d1)))
    a("v_sub_u32 %s, 32, %s" % (v(p), v(b)))
    a("v_cmp_eq_u32_e64 %s, 0, %s" % (sp(bz), v(b)))
    bitshift_left(a, [d0, d1], p, bz, 2, S_T)
    bitshift_left(a, un, p, bz, 10, S_T)
    # 3/2 reciprocal: dinv = floor((2^96 - 1) / d) - 2^32 from the 2/1
    # reciprocal of d1 (Algorithm 6)
    _reciprocal(a, d1, dinv)
    c1, ge = sp(S_T), sp(S_T + 2)
    a("v_mul_lo_u32 %s, %s, %s" % (v(p), v(d1), v(dinv)))
    a("v_add_co_u32 %s, %s, %s, %s" % (v(p), c1, v(p), v(d0)))         # p = d1 v + d0, carry
    a("v_cmp_ge_u32_e64 %s, %s, %s" % (ge, v(p), v(d1)))
    a("s_and_b64 %s, %s, %s" % (ge, ge, c1))
    a("v_subb_co_u32_e64 %s, %s, %s, 0, %s" % (v(dinv), sp(S_T + 4), v(dinv), c1))
    a("v_subb_co_u32_e64 %s, %s, %s, 0, %s" % (v(dinv), sp(S_T + 4), v(dinv), ge))
    a("v_cndmask_b32_e64 %s, 0, %s, %s" % (v(t0), v(d1), c1))
    a("v_sub_u32 %s, %s, %s" % (v(p), v(p), v(t0)))
    a("v_cndmask_b32_e64 %s, 0, %s, %s" % (v(t0), v(d1), ge))
    a("v_sub_u32 %s, %s, %s" % (v(p), v(p), v(t0)))
    a("v_mad_u64_u32 %s, %s, %s, %s, 0" % (vp(q0), sp(S_T + 6), v(dinv), v(d0)))   # (t1:t0) = v d0
    a("v_add_co_u32 %s, %s, %s, %s" % (v(q1), c1, v(p), v(q1)))       # p += t1, carry
    a("v_cmp_ge_u64_e64 %s, %s, %s" % (ge, vp(q0), dd))               # (p:t0) >= (d1:d0)
    a("s_and_b64 %s, %s, %s" % (ge, ge, c1))
    a("v_subb_co_u32_e64 %s, %s, %s, 0, %s" % (v(dinv), sp(S_T + 4), v(dinv), c1))
    a("v_subb_co_u32_e64 %s, %s, %s, 0, %s" % (v(dinv), sp(S_T + 4), v(dinv), ge))
    a("v_mov_b64 %s, %s" % (vp(r0), vp(R[0])))                         # r = un[9]:un[8] < d
    for j in reversed(range(8)):
        # (q1:q0) = dinv r1 + (r1:r0); r1' = r0 - q1 d1; (r1':r0') = (r1':u[j])
        # - d0 q1 - d; q1++; r1' >= q0: q1--, r' += d; r' >= d (unlikely):
        # q1++, r' -= d
        a("v_mad_u64_u32 %s, %s, %s, %s, %s" % (vp(q0), sp(S_T + 6), v(dinv), v(r1), vp(r0)))
        a("v_mul_lo_u32 %s, %s, %s" % (v(t1), v(q1), v(d1)))
        a("v_sub_u32 %s, %s, %s" % (v(r1), v(r0), v(t1)))
        a("v_mad_u64_u32 %s, %s, %s, %s, 0" % (vp(t0), sp(S_T + 6), v(d0), v(q1)))
        a("v_sub_co_u32 %s, vcc, %s, %s" % (v(r0), v(X[j]), v(t0)))
        a("v_subb_co_u32 %s, vcc, %s, %s, vcc" % (v(r1), v(r1), v(t1)))
        a("v_sub_co_u32 %s, vcc, %s, %s" % (v(r0), v(r0), v(d0)))
        a("v_subb_co_u32 %s, vcc, %s, %s, vcc" % (v(r1), v(r1), v(d1)))
        a("v_add_u32 %s, 1, %s" % (v(q1), v(q1)))
        a("v_cmp_ge_u32_e64 %s, %s, %s" % (ge, v(r1), v(q0)))
        a("v_subb_co_u32_e64 %s, %s, %s, 0, %s" % (v(R[j]), sp(S_T + 4), v(q1), ge))
        lab = exec_begin(a, S_T + 2, S_T)
        a("v_add_co_u32 %s, vcc, %s, %s" % (v(r0), v(r0), v(d0)))
        a("v_addc_co_u32 %s, vcc, %s, %s, vcc" % (v(r1), v(r1), v(d1)))
        exec_end(a, lab, S_T)
        a("v_cmp_ge_u64 vcc, %s, %s" % (vp(r0), dd))
        skip = a.uniq("d2s")
        a("s_cbranch_vccz %s" % skip)
        lab = exec_begin(a, None, S_T)
        a("v_add_u32 %s, 1, %s" % (v(R[j]), v(R[j])))
        a("v_sub_co_u32 %s, vcc, %s, %s" % (v(r0), v(r0), v(d0)))
        a("v_subb_co_u32 %s, vcc, %s, %s, vcc" % (v(r1), v(r1), v(d1)))
        exec_end(a, lab, S_T)
        a.label(skip)
    if want_rem:
        # remainder = r >> (b + 32 in the lanes that moved a limb)
        a("v_alignbit_b32 %s, %s, %s, %s" % (v(X[0]), v(r1), v(r0), v(b)))
        a("v_lshrrev_b32 %s, %s, %s" % (v(X[1]), v(b), v(r1)))
        lab = exec_begin(a, lq, S_T)
        moves(a, [X[0], X[1]], [X[1], None])
        exec_end(a, lab, S_T)
        moves(a, X[2:], [None] * 6)


def _reciprocal(a: Asm, d: int, dinv: int):
    """v[dinv] = floor((2^64-1)/d) - 2^32 for a normalised divisor v[d]
    (d >= 2^31) in every lane: f64 reciprocal, one Newton step (the estimate
    is then within one of the exact value), then one exact integer
    correction in each direction.  Clobbers T4..T9, s[S_T..S_T+7], vcc."""
    f0, f1, fe = T[4], T[6], T[8]
    a("v_cvt_f64_u32_e32 %s, %s" % (vp(f0), v(d)))
    a("v_rcp_f64_e32 %s, %s" % (vp(f1), vp(f0)))
    a("s_nop 1")
    a("v_fma_f64 %s, -%s, %s, 1.0" % (vp(fe), vp(f0), vp(f1)))            # e = 1 - d*r
    a("v_fma_f64 %s, %s, %s, %s" % (vp(f1), vp(f1), vp(fe), vp(f1)))      # r += r*e
    a("v_ldexp_f64 %s, %s, 64" % (vp(f1), vp(f1)))
    a("s_mov_b32 %s, 0" % s(S_T + 6))
    a("s_mov_b32 %s, 0xc1f00000" % s(S_T + 7))                          # -2^32
    a("v_add_f64 %s, %s, %s" % (vp(f1), vp(f1), sp(S_T + 6)))
    a("v_cvt_u32_f64_e32 %s, %s" % (v(dinv), vp(f1)))
    a("s_nop 1")
    p0, p1 = T[4], T[5]
    # p = dinv*d + (d << 32) = (2^32 + dinv) * d; carry -> too big
    a("v_mov_b32 %s, 0" % v(p0))
    a("v_mov_b32 %s, %s" % (v(p1), v(d)))
    a("v_mad_u64_u32 v[%d:%d], %s, %s, %s, v[%d:%d]" % (p0, p1, sp(S_T + 6), v(dinv), v(d), p0, p1))
    a("v_subb_co_u32_e64 %s, %s, %s, 0, %s" % (v(dinv), sp(S_T + 4), v(dinv), sp(S_T + 6)))
    # too small: (2^64-1) - p >= d  <=>  ~p_hi != 0 or ~p_lo >= d
    a("v_not_b32 %s, %s" % (v(p0), v(p0)))
    a("v_not_b32 %s, %s" % (v(p1), v(p1)))
    a("v_cmp_ne_u32_e64 %s, 0, %s" % (sp(S_T + 2), v(p1)))
    a("v_cmp_le_u32_e64 %s, %s, %s" % (sp(S_T), v(d), v(p0)))
    a("s_or_b64 %s, %s, %s" % (sp(S_T), sp(S_T), sp(S_T + 2)))
    a("s_andn2_b64 %s, %s, %s" % (sp(S_T), sp(S_T), sp(S_T + 6)))
    a("v_addc_co_u32_e64 %s, %s, %s, 0, %s" % (v(dinv), sp(S_T + 4), v(dinv), sp(S_T)))


def _div_digit(a: Asm, un, vn, j, d, dinv):
    """One quotient digit of Knuth D for every lane (see udivrem).
    Registers: A = T4:T5, P = T6:T7 (64-bit pairs), CR:RH = T8:T9 (RH = 0
    for the whole loop), QH = T11."""
    u2, u1 = un[j + 8], un[j + 7]
    A0, A1, P0, P1, CR, RH, QH = T[4], T[5], T[6], T[7], T[8], T[9], T[11]
    st = S_T
    lt = sp(st)                  # lanes with u2 < d (all but the u2 == d case)
    # 2-by-1 quotient via the reciprocal: qq = dinv * u2 + (u2:u1).  Lanes
    # with u2 == d (not < d) compute garbage here and take qhat = b - 1 below.
    # The addend is read in place when (u1, u2) is an aligned pair.
    a("v_cmp_lt_u32_e64 %s, %s, %s" % (lt, v(u2), v(d)))
    if u2 == u1 + 1 and u1 % 2 == 0:
        add = vp(u1)
    else:
        a("v_pk_mov_b32 %s, %s, %s op_sel:[%d,%d]" % (vp(A0), vp(u1 & ~1), vp(u2 & ~1), u1 & 1, u2 & 1))
        add = vp(A0)
    a("v_mad_u64_u32 v[%d:%d], %s, %s, %s, %s" % (A0, A1, sp(st + 6), v(dinv), v(u2), add))
    a("v_add_u32 %s, 1, %s" % (v(QH), v(A1)))                       # q1 (A0 = q0)
    a("v_mad_u64_u32 v[%d:%d], %s, %s, %s, 0" % (P0, P1, sp(st + 6), v(QH), v(d)))
    a("v_sub_u32 %s, %s, %s" % (v(CR), v(u1), v(P0)))                # r = u1 - q1*d
    a("v_cmp_gt_u32_e64 %s, %s, %s" % (sp(st + 2), v(CR), v(A0)))   # r > q0: q1--, r += d
    a("v_subb_co_u32_e64 %s, %s, %s, 0, %s" % (v(QH), sp(st + 4), v(QH), sp(st + 2)))
    a("v_cndmask_b32_e64 %s, 0, %s, %s" % (v(P0), v(d), sp(st + 2)))
    a("v_add_u32 %s, %s, %s" % (v(CR), v(CR), v(P0)))
    a("v_cmp_ge_u32_e64 %s, %s, %s" % (sp(st + 2), v(CR), v(d)))     # r >= d: q1++, r -= d
    a("v_addc_co_u32_e64 %s, %s, %s, 0, %s" % (v(QH), sp(st + 4), v(QH), sp(st + 2)))
    # lanes with u2 == d: qhat = b - 1.  qhat is now at most two above the
    # true digit (Knuth's Theorem B, normalised divisor); the add-back below
    # runs at most twice, and only for waves with a lane that needs it
    a("v_cndmask_b32_e64 %s, -1, %s, %s" % (v(QH), v(QH), lt))
    # multiply-subtract un[j..j+8] -= qh * vn as one borrow chain in vcc:
    # P = qh * vn[i] + carry (carry pair CR:RH with RH = 0), un[j+i] -= P.lo.
    # In line the chain covers digits 6, 7 only: enough when every lane with
    # qh != 0 has vn[0..5] == 0 (qh * 0 changes nothing); otherwise an out-of-
    # line chain from digit 4 (vn[0..3] == 0) or 0 runs instead.
    lab_wide, lab_full, lab_join = a.uniq("dmw"), a.uniq("dmf"), a.uniq("dmj")
    a("v_cmp_ne_u32_e64 %s, 0, %s" % (lt, v(QH)))
    a("s_andn2_b64 %s, %s, %s" % (sp(st + 2), lt, sp(DIV_Z6)))
    a("s_cbranch_scc1 %s" % lab_wide)

    def chain(first):
        for i in range(first, 8):
            add = "0" if i == first else "v[%d:%d]" % (CR, RH)
            a("v_mad_u64_u32 v[%d:%d], %s, %s, %s, %s" % (P0, P1, sp(st + 6), v(QH), v(vn[i]), add))
            a("v_mov_b32 %s, %s" % (v(CR), v(P1)))
            if i == first:
                a("v_sub_co_u32 %s, vcc, %s, %s" % (v(un[j + i]), v(un[j + i]), v(P0)))
            else:
                a("v_subb_co_u32 %s, vcc, %s, %s, vcc" % (v(un[j + i]), v(un[j + i]), v(P0)))
    chain(6)
    a.label(lab_join)
    a("v_subb_co_u32 %s, vcc, %s, %s, vcc" % (v(u2), v(u2), v(CR)))
    # borrow lanes went negative: quotient digit qh - 1 and add vn back under
    # exec (rare, out of line); without Knuth's test qh can be two too big:
    # lanes with no carry out of the first add-back take a second one
    a("s_mov_b64 %s, vcc" % sp(st + 4))
    a("v_subb_co_u32 %s, vcc, %s, 0, vcc" % (v(u2), v(QH)))       # digit into the dead top
    lab_ab, lab_x, lab_ret = a.uniq("dab"), a.uniq("dax"), a.uniq("dar")
    a("s_cmp_lg_u64 %s, 0" % sp(st + 4))
    a("s_cbranch_scc1 %s" % lab_ab)
    a.label(lab_ret)
    a.cold()
    a.label(lab_wide)
    a("s_andn2_b64 %s, %s, %s" % (sp(st + 2), lt, sp(DIV_Z4)))
    a("s_cbranch_scc1 %s" % lab_full)
    chain(4)
    a("s_branch %s" % lab_join)
    a.label(lab_full)
    chain(0)
    a("s_branch %s" % lab_join)
    a.label(lab_ab)
    a("s_mov_b64 %s, exec" % sp(st + 2))
    a("s_mov_b64 exec, %s" % sp(st + 4))
    for rnd in range(2):
        a("v_add_co_u32 %s, vcc, %s, %s" % (v(un[j]), v(un[j]), v(vn[0])))
        for i in range(1, 8):
            a("v_addc_co_u32 %s, vcc, %s, %s, vcc" % (v(un[j + i]), v(un[j + i]), v(vn[i])))
        if rnd == 0:
            a("s_andn2_b64 exec, exec, vcc")                        # still negative
            a("s_cbranch_execz %s" % lab_x)
            a("v_add_u32 %s, -1, %s" % (v(u2), v(u2)))
    a.label(lab_x)
    a("s_mov_b64 exec, %s" % sp(st + 2))
    a("s_branch %s" % lab_ret)
    a.hot()


def _cond_neg(a: Asm, regs: List[int], m: int):
    """regs = -regs in the lanes of s[m:m+1] (under exec; uses s[S_T+2:+3])."""
    lab = exec_begin(a, m, S_T + 2)
    a("v_sub_co_u32 %s, vcc, 0, %s" % (v(regs[0]), v(regs[0])))
    for j in range(1, 8):
        a("v_subb_co_u32 %s, vcc, 0, %s, vcc" % (v(regs[j]), v(regs[j])))
    exec_end(a, lab, S_T + 2)


DIV_CODE = {"UDIV": 0, "UREM": 1, "SDIV": 2, "SREM": 3, "SMOD": 4}


def body_div(a: Asm):
    """UDIV/UREM/SDIV/SREM/SMOD (op = S_VAR >> 4), SMT-LIB semantics."""
    NS, NT, Z, OPR = S_X, S_X + 2, S_X + 4, S_X + 6
    a.label(".Lbody_DIV_%=")
    heavy_prologue(a)
    a.read_slot(X, cur(F_A))
    a.read_slot(Y, cur(F_B))
    a("s_lshr_b32 %s, %s, 4" % (s(OPR), s(S_VAR)))
    lab_u = a.uniq("du")
    a("s_cmp_lt_u32 %s, 2" % s(OPR))
    a("s_cbranch_scc1 %s" % lab_u)
    lab_ns = a.uniq("dns")
    a("s_bitcmp1_b32 %s, 1" % s(S_VAR))
    a("s_cbranch_scc0 %s" % lab_ns)
    a("s_waitcnt lgkmcnt(0)")                          # the width masks (sext)
    sext(a, X, cur(F_W), S_M, T[0], S_T)
    sext(a, Y, cur(F_W), S_M, T[0], S_T)
    a.label(lab_ns)
    a("v_cmp_gt_i32_e64 %s, 0, %s" % (sp(NS), v(X[7])))
    a("v_cmp_gt_i32_e64 %s, 0, %s" % (sp(NT), v(Y[7])))
    _cond_neg(a, X, NS)
    _cond_neg(a, Y, NT)
    a.label(lab_u)
    lab_q, lab_dd = a.uniq("dq"), a.uniq("ddd")
    a("s_cmp_eq_u32 %s, 0" % s(OPR))
    a("s_cbranch_scc1 %s" % lab_q)
    a("s_cmp_eq_u32 %s, 2" % s(OPR))
    a("s_cbranch_scc1 %s" % lab_q)
    udivrem(a, want_rem=True, z=Z)
    a("s_branch %s" % lab_dd)
    a.label(lab_q)
    udivrem(a, want_rem=False, z=Z)
    a.label(lab_dd)
    # R = q, X = remainder (both 0 where the divisor is 0)
    labs = {k: a.uniq("dr%d" % k) for k in range(5)}
    lab_end = a.uniq("dre")
    for k in range(1, 5):
        a("s_cmp_eq_u32 %s, %d" % (s(OPR), k))
        a("s_cbranch_scc1 %s" % labs[k])
    def ones_where_zero():                             # R = z ? ~0 : R
        lab = exec_begin(a, Z, S_T + 2)
        for j in range(0, 8, 2):
            a("v_mov_b64 %s, -1" % vp(R[j]))
        exec_end(a, lab, S_T + 2)

    def rem_unless_zero(dst, src):                     # dst = z ? dst : src
        lab = exec_begin(a, Z, S_T + 2, invert=True)
        moves(a, dst, src)
        exec_end(a, lab, S_T + 2)

    def dividend_where_zero():                         # urem/srem/smod x/0 = x
        lab = exec_begin(a, Z, S_T + 2)
        a.read_slot(R, cur(F_A))                       # canonical at the width
        exec_end(a, lab, S_T + 2)

    a.label(labs[0])                                   # udiv: z ? ~0 : q
    ones_where_zero()
    a("s_branch %s" % lab_end)
    a.label(labs[1])                                   # urem: z ? x : rem
    rem_unless_zero(R, X)
    dividend_where_zero()
    a("s_branch %s" % lab_end)
    a.label(labs[2])                                   # sdiv
    ones_where_zero()
    a("s_xor_b64 %s, %s, %s" % (sp(NS), sp(NS), sp(NT)))
    _cond_neg(a, R, NS)
    a("s_branch %s" % lab_end)
    a.label(labs[3])                                   # srem: sign of the dividend
    rem_unless_zero(R, X)
    _cond_neg(a, R, NS)
    dividend_where_zero()
    a("s_branch %s" % lab_end)
    a.label(labs[4])                                   # smod: m = rem (X)
    a.read_slot(Y, cur(F_B))                           # t again
    lab_nx = a.uniq("dsx")
    a("s_bitcmp1_b32 %s, 1" % s(S_VAR))
    a("s_cbranch_scc0 %s" % lab_nx)
    sext(a, Y, cur(F_W), S_M, T[0], S_T)
    a.label(lab_nx)
    moves(a, R, X)                                     # base = ns ? -m : m
    _cond_neg(a, R, NS)
    a("s_xor_b64 %s, %s, %s" % (sp(NT), sp(NS), sp(NT)))               # ns != nt: + t
    lab = exec_begin(a, NT, S_T + 2)
    a("v_add_co_u32 %s, vcc, %s, %s" % (v(R[0]), v(R[0]), v(Y[0])))
    for j in range(1, 8):
        a("v_addc_co_u32 %s, vcc, %s, %s, vcc" % (v(R[j]), v(R[j]), v(Y[j])))
    exec_end(a, lab, S_T + 2)
    or_reduce(a, X, T[0])                              # m == 0 -> 0
    a("v_cmp_eq_u32 vcc, 0, %s" % v(T[0]))
    lab = exec_begin(a, None, S_T + 2)
    moves(a, R, [None] * 8)
    exec_end(a, lab, S_T + 2)
    dividend_where_zero()
    a.label(lab_end)
    heavy_finish(a, R)
    a.flush_cold()


# ---------------------------------------------------------------------------
# the whole interpreter
# ---------------------------------------------------------------------------

CHEAP = {
    "NOP": h_nop, "HALT": h_halt, "CONST": h_const, "LEAF": h_leaf,
    "RELOAD_SCR": h_reload_scr, "ADD": h_add, "SUB": h_sub, "AND": h_and, "OR": h_or,
    "XOR": h_xor, "NOT": h_not, "EQ": h_eq, "ULT": h_ult, "ULE": h_ule, "SLT": h_slt,
    "SLE": h_sle, "ITE": h_ite, "CONCAT": h_concat, "EXTRACT": h_extract, "SEXT": h_sext,
    "NEG": h_neg, "OUT": h_out, "ROOT": h_root, "MOV": h_mov, "SUBR": h_subr, "ITEN": h_iten,
    "WAITVM": h_waitvm, "MUL": h_mul, "BCAST": h_bcast, "CDWE": h_cdwe, "CDWX": h_cdwx,
    "SHL": h_shift("SHL"), "LSHR": h_shift("LSHR"), "ASHR": h_shift("ASHR"),
}
SLOT_HANDLERS = {"SPILL_LDS": h_spill_lds, "SPILL_SCR": h_spill_scr, "RELOAD_LDS": h_reload_lds}
HEAVY = {"UMULNO": "UMULNO",
         "UDIV": "DIV", "UREM": "DIV", "SDIV": "DIV", "SREM": "DIV", "SMOD": "DIV"}
HEAVY_AOPS = sorted(AOP[n] for n in HEAVY)


def emit_handler(a: Asm, name: str, var: int, bank: int) -> None:
    """The handler of family ``name``, variant ``var``, record bank ``bank``
    (its body only; the caller places the label)."""
    root_v, mask_v = bool(var & V_ROOT), bool(var & V_MASK)
    dc_v, w32_v, ip_v = bool(var & V_DC), bool(var & V_W32), bool(var & V_IP)
    a.nw = bool(var & V_NW)
    if name == "LEAFD":
        h_leafd(a, bank, var)
    elif name == "RELOADD":
        h_reloadd(a, bank, var)
    elif name in SLOT_VARIANT:
        SLOT_HANDLERS[name](a, bank, var)
    elif name == "EQSEL":
        h_eqsel(a, bank, var)
    elif name == "EXTRACTN":
        h_extractn(a, bank, var)
    elif name == "CONCATQ":
        h_concatq(a, bank, var)
    elif name in CHEAP:
        CHEAP[name](a, bank, root_v, mask_v, dc_v, w32_v, ip_v)
    else:
        bits = var | (DIV_CODE.get(name, 0) << 4)
        heavy_stub(a, bank, bits, ".Lbody_%s_%%=" % HEAVY[name])
    a.nw = False


def generate() -> List[str]:
    a = Asm()
    a("s_mov_b32 %s, m0" % s(S_M0))
    load_sm64_consts(a)
    # mg_pdesc: code@0 consts@8 gen@16 ... xcode@48 btab@56 jit@64
    a("s_load_dwordx2 %s, %s, 0x%x" % (sp(S_CONST), IN["desc"], PDESC_CONSTS))
    a("s_load_dwordx2 %s, %s, 0x%x" % (sp(S_CODE), IN["desc"], PDESC_XCODE))
    a("s_load_dwordx2 %s, %s, 0x%x" % (sp(S_JMP), IN["desc"], PDESC_JIT))
    a("v_mov_b32 %s, 1" % OP_ROOT)
    a("s_getpc_b64 %s" % sp(S_BASE))
    a.label(".Lbase_%=")
    a("s_bitcmp1_b32 %s, 1" % IN["mode"])
    a("s_cbranch_scc1 .Lquery_%=")
    a("s_mov_b32 %s, 32" % s(S_IP))
    a("s_waitcnt lgkmcnt(0)")
    # a compiled program (mythril_amd/jit.py) runs instead of the records
    a("s_cmp_lg_u64 %s, 0" % sp(S_JMP))
    a("s_cbranch_scc1 .Ljit_%=")
    a("s_load_dwordx8 s[%d:%d], %s, 0x0" % (BANK[0], BANK[0] + 7, sp(S_CODE)))
    dispatch(a, 0)
    # compiled program: call it (it returns through s[JIT_RET]), then the
    # dispatch base is re-established for the far jump to the exit
    a.label(".Ljit_%=")
    a("s_swappc_b64 %s, %s" % (sp(JIT_RET), sp(S_JMP)))
    a("s_getpc_b64 %s" % sp(S_BASE))
    a.label(".Ljret_%=")
    a("s_sub_u32 %s, %s, (.Ljret_%%= - .Lbase_%%=)" % (s(S_BASE), s(S_BASE)))
    a("s_subb_u32 %s, %s, 0" % (s(S_BASE + 1), s(S_BASE + 1)))
    far_jump(a, ".Lexit_%=")
    # query mode: table[h] = offset of handler h from .Lbase
    a.label(".Lquery_%=")
    a("s_waitcnt lgkmcnt(0)")              # the descriptor loads (S_JMP is reused)
    a("v_mov_b32 %s, 0" % v(T[0]))
    a("s_mov_b64 %s, %s" % (sp(S_T), IN["table"]))
    for h in range(NUM_HANDLERS):
        if h and h % 512 == 0:
            a("s_add_u32 %s, %s, 2048" % (s(S_T), s(S_T)))
            a("s_addc_u32 %s, %s, 0" % (s(S_T + 1), s(S_T + 1)))
        a("v_mov_b32 %s, (.Lh%d_%%= - .Lbase_%%=)" % (v(T[1]), canonical(h)))
        a("global_store_dword %s, %s, %s offset:%d" % (v(T[0]), v(T[1]), sp(S_T), 4 * (h % 512)))
    a("s_waitcnt vmcnt(0)")
    far_jump(a, ".Lexit_%=")
    for name in AOPS:
        aop = AOP[name]
        for var in range(NVAR):
            if canon_var(name, var) != var:
                continue
            for bank in (0, 1):
                a.label(".Lh%d_%%=" % hid(aop, var, bank))
                emit_handler(a, name, var, bank)
        # a shared body right after the stubs that branch to it (s_branch
        # reaches +-128 KB; at the end of the handlers the division body was
        # within 3 % of that from its first stub); handlers end in a
        # dispatch, so nothing falls into a body
        if name == "SMOD":
            body_div(a)
        elif name == "UMULNO":
            body_umulno(a)
    a.label(".Lexit_%=")
    a("s_set_gpr_idx_off")
    a("s_mov_b32 m0, %s" % s(S_M0))
    return drop_redundant_idx_off(a.lines)


def drop_redundant_idx_off(lines: List[str]) -> List[str]:
    """Remove every s_set_gpr_idx_off after which each path reaches an
    s_set_gpr_idx_on (it sets index and mode in any state) or a dispatch
    (the next handler turns the mode off lazily, Asm.__call__) before any
    instruction that touches VGPRs.  A path reaching another off, an
    s_set_gpr_idx_idx / _mode or the end keeps the off (conservative)."""
    body = [l.strip() for l in lines]
    label_at = {t[:-1]: i for i, t in enumerate(body) if t.endswith(":")}

    def succ(i: int) -> List[int]:
        t = body[i]
        op = t.split(None, 1)[0] if t else ""
        if op == "s_setpc_b64":
            return []
        if op == "s_branch":
            return [label_at[t.split()[1]]]
        if op.startswith("s_cbranch"):
            return [label_at[t.split()[1]], i + 1]
        return [i + 1]

    def redundant(i: int) -> bool:
        stack, seen = [i + 1], set()
        while stack:
            j = stack.pop()
            if j in seen:
                continue
            seen.add(j)
            if j >= len(body):
                return False
            t = body[j]
            if not t or t.endswith(":") or t.startswith("."):
                stack.append(j + 1)
                continue
            op = t.split(None, 1)[0]
            if op.startswith("s_set_gpr_idx_on"):
                continue
            if op.startswith("s_set_gpr_idx_"):
                return False
            if op == "s_setpc_b64":
                continue                          # next handler: lazy off
            if not op.startswith("s_"):
                return False                      # a VGPR access
            stack.extend(succ(j))
        return True

    drop = {i for i, t in enumerate(body) if t == "s_set_gpr_idx_off" and redundant(i)}
    return [l for i, l in enumerate(lines) if i not in drop]


def operand_constraints() -> Dict[str, str]:
    """Inline-asm constraint of every operand: its pinned register."""
    out = {}
    for k, r in PINNED.items():
        out[k] = ("={%s}" if k == "root" else "{%s}") % r
    return out


def clobbers() -> List[str]:
    vs = ['"v%d"' % i for i in range(NVGPR_FIXED)]
    ss = ['"s%d"' % i for i in range(BANK[0], S_LAST + 1)]
    # m0 is saved/restored inside; exec is restored on every path
    return vs + ss + ['"vcc"', '"scc"', '"memory"']


def digest(lines: Optional[List[str]] = None) -> str:
    """Short hash of the generated assembly and its operand registers
    (embedded in the library, so a stale build is detected:
    engine.load_library, tests/test_abi.py)."""
    import hashlib
    text = list(lines or generate()) + ["%s=%s" % kv for kv in sorted(PINNED.items())]
    return hashlib.sha256("\n".join(text).encode()).hexdigest()[:16]


def write_outputs(csrc: str) -> None:
    lines = generate()
    body = " \\\n".join('"%s\\n"' % l.replace('"', '\\"') for l in lines)
    oc = operand_constraints()
    cons = "".join('#define MG_ASM_C_%s "%s"\n' % (k.upper(), c) for k, c in oc.items())
    inc = ("// GENERATED by mythril_amd/asmgen.py -- do not edit.\n"
           "// Inline-asm body of mg_interp_asm (gfx950), %d lines.\n"
           "#define MG_ASM_BODY \\\n%s\n\n"
           "#define MG_ASM_CLOBBERS %s\n"
           "// operand registers (asmgen.PINNED; compiled programs use them too)\n%s"
           "#define MG_ASM_DIGEST \"%s\"\n") % (len(lines), body, ", ".join(clobbers()), cons,
                                                 digest(lines))
    _write_if_changed(os.path.join(csrc, "mg_interp_gfx950.inc"), inc)
    hdr = ["// GENERATED by mythril_amd/asmgen.py -- do not edit.",
           "#ifndef MG_ASM_HANDLERS_H", "#define MG_ASM_HANDLERS_H",
           "#define MGA_NUM_HANDLERS %d" % NUM_HANDLERS,
           "#define MGA_NVAR %d" % NVAR,
           "#define MGA_V_ROOT %d" % V_ROOT, "#define MGA_V_MASK %d" % V_MASK,
           "#define MGA_V_DC %d" % V_DC, "#define MGA_V_W32 %d" % V_W32,
           "#define MGA_V_IP %d" % V_IP, "#define MGA_V_NW %d" % V_NW,
           "#define MGA_V_WAITD %d" % V_WAITD,
           "#define MGA_V_NARROW %d" % V_NARROW,
           "#define MGA_V_NEG %d" % V_NEG, "#define MGA_V_GEN %d" % V_GEN,
           "#define MGA_HID(aop, var, bank) ((((aop) * MGA_NVAR) + (var)) * 2 + (bank))",
           "#define MGA_FB %d" % FB, "#define MGA_NREG %d" % NREG,
           "enum mga_op {"]
    hdr += ["    MGA_%s = %d," % (n, i) for i, n in enumerate(AOPS)]
    hdr += ["    MGA_NUM_OPS = %d" % len(AOPS), "};",
            "/* heavy ops always prefetch the next record into bank A */",
            "static inline int mga_is_heavy(int aop) {",
            "    return " + " || ".join("aop == %d" % x for x in HEAVY_AOPS) + ";", "}",
            "#endif", ""]
    _write_if_changed(os.path.join(csrc, "mg_asm_handlers.h"), "\n".join(hdr))


def _write_if_changed(path: str, text: str) -> None:
    if os.path.exists(path):
        with open(path) as fh:
            if fh.read() == text:
                return
    with open(path, "w") as fh:
        fh.write(text)


if __name__ == "__main__":
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc")
    write_outputs(here)
    print("wrote", here)
