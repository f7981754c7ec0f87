"""TEST INFRASTRUCTURE — instruction-level simulator of the generated gfx950
assembly interpreter (mythril_amd/asmgen.py), one wave of 64 lanes.

It executes the exact text that goes into the inline asm, so handler logic,
GPR-index usage, carries and lane masks are checked on the CPU before any
GPU run.  Loads complete at the matching ``s_waitcnt`` (SMEM and LDS at
lgkmcnt(0), VMEM/scratch at vmcnt(0)); reading or overwriting a register
whose load is still pending is an error, so a missing wait is caught.
``v_rcp_f64`` can be perturbed to exercise the reciprocal correction.

Only the instructions the generator emits are implemented; anything else
raises.  Semantics follow the CDNA3/4 ISA (gfx950).
"""

from __future__ import annotations

import re
import struct
from typing import Dict, List, Optional, Tuple

import numpy as np

M32 = 0xFFFFFFFF
M64 = (1 << 64) - 1
NL = 64
CODE_BASE = 0x7F0000000000
LANES = np.arange(NL)


class SimError(Exception):
    pass


def _mask_to_bool(m: int) -> np.ndarray:
    return ((m >> LANES.astype(np.uint64)) & 1).astype(bool) if False else \
        np.array([(m >> i) & 1 for i in range(NL)], dtype=bool)


def _bool_to_mask(b: np.ndarray) -> int:
    m = 0
    for i in np.flatnonzero(b):
        m |= 1 << int(i)
    return m


class Memory:
    """Flat 64-bit address space made of named regions."""

    def __init__(self):
        self.regions: List[Tuple[int, bytearray, str]] = []
        self.next = 0x10000000

    def alloc(self, data: bytes, name: str, align: int = 256) -> int:
        base = self.next
        buf = bytearray(data)
        self.regions.append((base, buf, name))
        self.next = base + ((len(buf) + 4096 + align) // align) * align
        return base

    def _find(self, addr: int, n: int):
        for base, buf, name in self.regions:
            if base <= addr and addr + n <= base + len(buf):
                return buf, addr - base
        raise SimError("memory access out of bounds: 0x%x (+%d)" % (addr, n))

    def read32(self, addr: int) -> int:
        buf, off = self._find(addr, 4)
        return struct.unpack_from("<I", buf, off)[0]

    def write32(self, addr: int, val: int):
        buf, off = self._find(addr, 4)
        struct.pack_into("<I", buf, off, val & M32)

    def region(self, base: int) -> bytearray:
        for b, buf, _ in self.regions:
            if b == base:
                return buf
        raise KeyError(base)


_TOK = re.compile(r"\s*([^,]+\([^)]*\)|[^,]+)\s*(?:,|$)")


def _split_ops(s: str) -> List[str]:
    out = []
    pos = 0
    mo = re.search(r"\s+(op_sel:\[\d,\d\])\s*$", s)      # VOP3P modifier (has a comma)
    if mo:
        return _split_ops(s[:mo.start()]) + [mo.group(1)]
    while pos < len(s):
        m = _TOK.match(s, pos)
        if not m or m.end() == pos:
            break
        tok = m.group(1).strip()
        mm = re.fullmatch(r"(.*\S)\s+(offset:\d+|clamp)", tok)
        if mm:
            out.extend([mm.group(1), mm.group(2)])
        else:
            out.append(tok)
        pos = m.end()
    return [o for o in out if o]


class Wave:
    def __init__(self, lines: List[str], subst: Dict[str, str], mem: Memory,
                 rcp_noise: float = 0.0, seed: int = 0):
        self.mem = mem
        self.rcp_noise = rcp_noise
        self.rng = np.random.default_rng(seed)
        self.instrs: List[Tuple[str, List[str], str]] = []
        self.labels: Dict[str, int] = {}
        for raw in lines:
            text = raw.strip()
            for k, val in subst.items():
                text = text.replace(k, val)
            text = text.replace("%=", "0")
            if not text or text.startswith(".p2align"):   # layout only
                continue
            if text.endswith(":"):
                self.labels[text[:-1]] = len(self.instrs)
                continue
            parts = text.split(None, 1)
            self.instrs.append((parts[0], _split_ops(parts[1]) if len(parts) > 1 else [], text))
        self.s = [0] * 128
        self.v = np.zeros((256, NL), dtype=np.uint64)
        self.vcc = 0
        self.exec = (1 << NL) - 1
        self.scc = 0
        self.m0 = 0
        self.idx_on = False
        self.idx_mode = set()
        self.pending: Dict[Tuple[str, int], Tuple[str, object]] = {}
        self.lds = bytearray(160 * 1024)
        self.scratch = [bytearray(4096) for _ in range(NL)]
        self.count = 0

    # ---- operand helpers --------------------------------------------------
    def _check(self, key):
        if key in self.pending:
            raise SimError("register %s%d read/overwritten while its load is pending" % key)

    def sreg(self, name: str) -> Tuple[int, int]:
        """-> (first index, count) for s-registers, or special."""
        m = re.fullmatch(r"s(\d+)", name)
        if m:
            return int(m.group(1)), 1
        m = re.fullmatch(r"s\[(\d+):(\d+)\]", name)
        if m:
            a, b = int(m.group(1)), int(m.group(2))
            return a, b - a + 1
        raise SimError("not an sgpr: " + name)

    def sread(self, op: str, width: int = 32) -> int:
        op = op.strip()
        if op == "vcc":
            return self.vcc
        if op == "exec":
            return self.exec
        if op == "m0":
            return self.m0
        if op.startswith("s"):
            a, n = self.sreg(op)
            val = 0
            for i in range(n):
                self._check(("s", a + i))
                val |= self.s[a + i] << (32 * i)
            return val
        return self._const(op, width)

    def swrite(self, op: str, val: int):
        op = op.strip()
        if op == "vcc":
            self.vcc = val & M64
            return
        if op == "exec":
            self.exec = val & M64
            return
        if op == "m0":
            self.m0 = val & M32
            return
        a, n = self.sreg(op)
        for i in range(n):
            self._check(("s", a + i))
            self.s[a + i] = (val >> (32 * i)) & M32

    def _const(self, op: str, width: int = 32) -> int:
        op = op.strip()
        m = re.fullmatch(r"\((\.L\S+) - (\.L\S+)\)", op)
        if m:
            return (8 * (self.labels[m.group(1)] - self.labels[m.group(2)])) & M32
        if op == "1.0":
            return 0x3FF0000000000000 if width == 64 else 0x3F800000
        try:
            x = int(op, 0)
        except ValueError:
            raise SimError("bad operand " + op)
        return x & (M64 if width == 64 else M32)

    def vidx(self, op: str, pos: Optional[str], is_valu: bool) -> Tuple[int, int]:
        m = re.fullmatch(r"v(\d+)", op)
        if m:
            a, n = int(m.group(1)), 1
        else:
            m = re.fullmatch(r"v\[(\d+):(\d+)\]", op)
            if not m:
                raise SimError("not a vgpr: " + op)
            a, n = int(m.group(1)), int(m.group(2)) - int(m.group(1)) + 1
        if is_valu and self.idx_on and pos in self.idx_mode:
            a += self.m0 & 0xFF
        if a + n > 256:
            raise SimError("vgpr out of range v%d" % (a + n - 1))
        return a, n

    def vread(self, op: str, pos: Optional[str] = None, width: int = 32, valu=True) -> np.ndarray:
        op = op.strip()
        neg = False
        if op.startswith("-v"):
            neg, op = True, op[1:]
        if op.startswith("v"):
            a, n = self.vidx(op, pos, valu)
            for i in range(n):
                self._check(("v", a + i))
            val = self.v[a].copy()
            if n == 2:
                val = val | (self.v[a + 1] << np.uint64(32))
            if neg:
                val = val ^ np.uint64(1 << 63)      # f64 negation modifier
            return val
        if op.startswith("s") or op in ("vcc", "exec", "m0"):
            x = self.sread(op, width)
            return np.full(NL, x, dtype=np.uint64)
        return np.full(NL, self._const(op, width), dtype=np.uint64)

    def vwrite(self, op: str, val: np.ndarray, pos: str = "DST", valu=True, mask=None):
        a, n = self.vidx(op.strip(), pos, valu)
        act = _mask_to_bool(self.exec) if mask is None else mask
        val = np.asarray(val, dtype=np.uint64)
        for i in range(n):
            self._check(("v", a + i))
            part = (val >> np.uint64(32 * i)) & np.uint64(M32)
            self.v[a + i] = np.where(act, part, self.v[a + i])

    def lanes_mask(self, op: str) -> np.ndarray:
        return _mask_to_bool(self.sread(op, 64))

    def wr_lanes(self, op: str, b: np.ndarray):
        self.swrite(op, _bool_to_mask(b & _mask_to_bool(self.exec)))

    # ---- pending loads -----------------------------------------------------
    def _defer(self, kind: str, key, apply, lanes=None):
        """Queue a load's register write until its counter is waited for.
        Two outstanding vector-memory loads may target one register only
        with disjoint lane sets (VMEM returns in issue order, so the writes
        then commute); anything else is an error."""
        if key in self.pending:
            kd, prev, plan = self.pending[key]
            if not (kind == kd == "vm" and lanes is not None and plan is not None
                    and not np.any(lanes & plan)):
                raise SimError("overlapping pending loads into %s%d" % key)

            def both(prev=prev, apply=apply):
                prev()
                apply()
            self.pending[key] = (kind, both, plan | lanes)
            return
        self.pending[key] = (kind, apply, lanes)

    def _wait(self, kind: str):
        for key in [k for k, (kd, _, _) in self.pending.items() if kd == kind]:
            _, apply, _ = self.pending.pop(key)
            apply()

    # ---- execution -----------------------------------------------------------
    def addr_of(self, label: str) -> int:
        return CODE_BASE + 8 * self.labels[label]

    def run(self, max_steps: int = 2_000_000):
        pc = 0
        while True:
            if pc >= len(self.instrs):
                return
            self.count += 1
            if self.count > max_steps:
                raise SimError("step limit (infinite loop?)")
            op, args, text = self.instrs[pc]
            try:
                nxt = self.step(op, args, pc)
            except SimError as e:
                raise SimError("%s  [at %d: %s]" % (e, pc, text))
            pc = pc + 1 if nxt is None else nxt

    def _target(self, label: str) -> int:
        if label not in self.labels:
            raise SimError("unknown label " + label)
        return self.labels[label]

    def step(self, op: str, a: List[str], pc: int):
        base = op.replace("_e32", "").replace("_e64", "")
        if base.startswith("s_") or base in ("scratch_store_dwordx4", "scratch_load_dwordx4"):
            pass
        return getattr(self, "i_" + base, self._unknown(base))(a, pc)

    def _unknown(self, base):
        def f(a, pc):
            raise SimError("unimplemented instruction " + base)
        return f

    # ---------------- SALU / control ----------------
    def i_s_nop(self, a, pc):
        return None

    def i_s_endpgm(self, a, pc):
        return len(self.instrs)          # the C++ shell's code after the asm

    def i_s_waitcnt(self, a, pc):
        t = " ".join(a)
        if "lgkmcnt(0)" in t:
            self._wait("lgkm")
        if "vmcnt(0)" in t:
            self._wait("vm")
        return None

    def i_s_mov_b32(self, a, pc):
        self.swrite(a[0], self.sread(a[1]))

    def i_s_mov_b64(self, a, pc):
        self.swrite(a[0], self.sread(a[1], 64))

    def _sop2(self, a, f, width=32, setscc="nz"):
        x, y = self.sread(a[1], width), self.sread(a[2], width)
        mask = M32 if width == 32 else M64
        r = f(x, y) & mask
        self.swrite(a[0], r)
        if setscc == "nz":
            self.scc = int(r != 0)

    def i_s_add_u32(self, a, pc):
        x, y = self.sread(a[1]), self.sread(a[2])
        r = x + y
        self.swrite(a[0], r & M32)
        self.scc = int(r >> 32)

    def i_s_addc_u32(self, a, pc):
        x, y = self.sread(a[1]), self.sread(a[2])
        r = x + y + self.scc
        self.swrite(a[0], r & M32)
        self.scc = int(r >> 32)

    def i_s_sub_u32(self, a, pc):
        x, y = self.sread(a[1]), self.sread(a[2])
        self.swrite(a[0], (x - y) & M32)
        self.scc = int(x < y)

    def i_s_subb_u32(self, a, pc):
        x, y = self.sread(a[1]), self.sread(a[2])
        r = x - y - self.scc
        self.swrite(a[0], r & M32)
        self.scc = int(r < 0)

    def i_s_and_b32(self, a, pc):
        self._sop2(a, lambda x, y: x & y)

    def i_s_bfe_u32(self, a, pc):
        # S1[4:0] = offset, S1[22:16] = width
        self._sop2(a, lambda x, y: (x >> (y & 31)) & ((1 << ((y >> 16) & 0x7F)) - 1))

    def i_s_xor_b32(self, a, pc):
        self._sop2(a, lambda x, y: x ^ y)

    def i_s_and_b64(self, a, pc):
        self._sop2(a, lambda x, y: x & y, 64)

    def i_s_or_b64(self, a, pc):
        self._sop2(a, lambda x, y: x | y, 64)

    def i_s_xor_b64(self, a, pc):
        self._sop2(a, lambda x, y: x ^ y, 64)

    def i_s_andn2_b64(self, a, pc):
        self._sop2(a, lambda x, y: x & ~y, 64)

    def i_s_and_saveexec_b64(self, a, pc):
        m = self.sread(a[1], 64)
        self.swrite(a[0], self.exec)
        self.exec = m & self.exec
        self.scc = int(self.exec != 0)

    def i_s_andn1_saveexec_b64(self, a, pc):
        m = self.sread(a[1], 64)
        self.swrite(a[0], self.exec)
        self.exec = ~m & self.exec & M64
        self.scc = int(self.exec != 0)

    def i_s_lshl_b32(self, a, pc):
        self._sop2(a, lambda x, y: x << (y & 31))

    def i_s_lshr_b32(self, a, pc):
        self._sop2(a, lambda x, y: x >> (y & 31))

    def i_s_lshr_b64(self, a, pc):
        x, y = self.sread(a[1], 64), self.sread(a[2])
        r = x >> (y & 63)
        self.swrite(a[0], r)
        self.scc = int(r != 0)

    def i_s_lshl_b64(self, a, pc):
        x, y = self.sread(a[1], 64), self.sread(a[2])
        r = (x << (y & 63)) & M64
        self.swrite(a[0], r)
        self.scc = int(r != 0)

    def i_s_mul_i32(self, a, pc):
        self.swrite(a[0], (self.sread(a[1]) * self.sread(a[2])) & M32)

    def i_s_mul_hi_u32(self, a, pc):
        self.swrite(a[0], (self.sread(a[1]) * self.sread(a[2])) >> 32)

    def i_s_cmp_eq_u32(self, a, pc):
        self.scc = int(self.sread(a[0]) == self.sread(a[1]))

    def i_s_cmp_lg_u32(self, a, pc):
        self.scc = int(self.sread(a[0]) != self.sread(a[1]))

    def i_s_cmp_lt_u32(self, a, pc):
        self.scc = int(self.sread(a[0]) < self.sread(a[1]))

    def i_s_cmp_eq_u64(self, a, pc):
        self.scc = int(self.sread(a[0], 64) == self.sread(a[1], 64))

    def i_s_cmp_lg_u64(self, a, pc):
        self.scc = int(self.sread(a[0], 64) != self.sread(a[1], 64))

    def i_s_cselect_b32(self, a, pc):
        self.swrite(a[0], self.sread(a[1]) if self.scc else self.sread(a[2]))

    def i_s_cselect_b64(self, a, pc):
        self.swrite(a[0], self.sread(a[1], 64) if self.scc else self.sread(a[2], 64))

    def i_s_bitcmp1_b32(self, a, pc):
        self.scc = (self.sread(a[0]) >> (self.sread(a[1]) & 31)) & 1

    def i_s_branch(self, a, pc):
        return self._target(a[0])

    def i_s_cbranch_scc0(self, a, pc):
        return self._target(a[0]) if not self.scc else None

    def i_s_cbranch_scc1(self, a, pc):
        return self._target(a[0]) if self.scc else None

    def i_s_cbranch_vccz(self, a, pc):
        return self._target(a[0]) if self.vcc == 0 else None

    def i_s_cbranch_vccnz(self, a, pc):
        return self._target(a[0]) if self.vcc != 0 else None

    def i_s_cbranch_execz(self, a, pc):
        return self._target(a[0]) if self.exec == 0 else None

    def i_s_cbranch_execnz(self, a, pc):
        return self._target(a[0]) if self.exec != 0 else None

    def i_s_getpc_b64(self, a, pc):
        self.swrite(a[0], CODE_BASE + 8 * (pc + 1))

    def i_s_setpc_b64(self, a, pc):
        t = self.sread(a[0], 64)
        off = t - CODE_BASE
        if off < 0 or off % 8 or off // 8 >= len(self.instrs):
            raise SimError("s_setpc to a non-instruction address 0x%x" % t)
        return off // 8

    def i_s_swappc_b64(self, a, pc):
        t = self.sread(a[1], 64)
        self.swrite(a[0], CODE_BASE + 8 * (pc + 1))
        off = t - CODE_BASE
        if off < 0 or off % 8 or off // 8 >= len(self.instrs):
            raise SimError("s_swappc to a non-instruction address 0x%x" % t)
        return off // 8

    def i_s_set_gpr_idx_on(self, a, pc):
        self.m0 = (self.m0 & ~0xFF) | (self.sread(a[0]) & 0xFF)
        self.idx_mode = set(re.search(r"gpr_idx\(([^)]*)\)", a[1]).group(1).split(","))
        self.idx_on = True

    def i_s_set_gpr_idx_idx(self, a, pc):
        self.m0 = (self.m0 & ~0xFF) | (self.sread(a[0]) & 0xFF)

    def i_s_set_gpr_idx_mode(self, a, pc):
        self.idx_mode = set(re.search(r"gpr_idx\(([^)]*)\)", a[0]).group(1).split(","))

    def i_s_set_gpr_idx_off(self, a, pc):
        self.idx_on = False

    def i_s_load_dwordx2(self, a, pc):
        self._sload(a, 2)

    def i_s_load_dwordx8(self, a, pc):
        self._sload(a, 8)

    def _sload(self, a, n):
        dst, _ = self.sreg(a[0])
        base = self.sread(a[1], 64)
        off = self.sread(a[2]) if a[2].startswith("s") else int(a[2], 0)
        addr = (base + off) & M64
        vals = [self.mem.read32(addr + 4 * i) for i in range(n)]
        for i in range(n):
            def apply(i=i):
                self.s[dst + i] = vals[i]
            self._defer("lgkm", ("s", dst + i), apply)

    # ---------------- VALU ----------------
    def _act(self):
        return _mask_to_bool(self.exec)

    def i_v_mov_b32(self, a, pc):
        self.vwrite(a[0], self.vread(a[1], "SRC0"))

    def i_v_mov_b64(self, a, pc):
        self.vwrite(a[0], self.vread(a[1], "SRC0", 64))

    def i_v_readfirstlane_b32(self, a, pc):
        # the lowest active lane (lane 0 with exec = 0)
        x = self.vread(a[1], "SRC0")
        lane = (self.exec & -self.exec).bit_length() - 1 if self.exec else 0
        self.swrite(a[0], int(x[lane]) & M32)

    def _vop2(self, a, f):
        x = self.vread(a[1], "SRC0")
        y = self.vread(a[2], "SRC1")
        self.vwrite(a[0], f(x, y) & np.uint64(M32))

    def i_v_and_b32(self, a, pc):
        self._vop2(a, lambda x, y: x & y)

    def i_v_or_b32(self, a, pc):
        self._vop2(a, lambda x, y: x | y)

    def i_v_xor_b32(self, a, pc):
        self._vop2(a, lambda x, y: x ^ y)

    def i_v_add_u32(self, a, pc):
        if a and a[-1] == "clamp":
            x, y = self.vread(a[1], "SRC0"), self.vread(a[2], "SRC1")
            self.vwrite(a[0], np.minimum(x + y, np.uint64(M32)))
            return
        self._vop2(a, lambda x, y: x + y)

    def i_v_sub_u32(self, a, pc):
        self._vop2(a, lambda x, y: x - y)

    def i_v_subrev_u32(self, a, pc):
        self._vop2(a, lambda x, y: y - x)

    def i_v_mul_lo_u32(self, a, pc):
        self._vop2(a, lambda x, y: (x * y) & np.uint64(M32))

    def i_v_mul_hi_u32(self, a, pc):
        self._vop2(a, lambda x, y: (x * y) >> np.uint64(32))

    def i_v_lshlrev_b32(self, a, pc):
        self._vop2(a, lambda s, x: x << (s & np.uint64(31)))

    def i_v_lshrrev_b32(self, a, pc):
        self._vop2(a, lambda s, x: x >> (s & np.uint64(31)))

    def i_v_ashrrev_i32(self, a, pc):
        s = self.vread(a[1], "SRC0") & np.uint64(31)
        x = self.vread(a[2], "SRC1").astype(np.uint32).view(np.int32).astype(np.int64)
        r = (x >> s.astype(np.int64)).astype(np.int64) & M32
        self.vwrite(a[0], r.astype(np.uint64))

    def i_v_not_b32(self, a, pc):
        self.vwrite(a[0], (~self.vread(a[1], "SRC0")) & np.uint64(M32))

    def i_v_ffbh_u32(self, a, pc):
        x = self.vread(a[1], "SRC0")
        r = np.array([(32 - int(t).bit_length()) if t else M32 for t in x], dtype=np.uint64)
        self.vwrite(a[0], r)

    def _vop3(self, a, f, n):
        srcs = [self.vread(a[1 + i], "SRC%d" % i) for i in range(n)]
        self.vwrite(a[0], f(*srcs) & np.uint64(M32))

    def i_v_pk_mov_b32(self, a, pc):
        """dst.lo = src0 half op_sel[0], dst.hi = src1 half op_sel[1]."""
        sel = [int(x) for x in re.findall(r"\d", a[3])] if len(a) > 3 else [0, 0]
        halves = []
        for k, src in enumerate((a[1], a[2])):
            val = self.vread(src, "SRC%d" % k, 64)
            halves.append((val >> np.uint64(32 * sel[k])) & np.uint64(M32))
        self.vwrite(a[0], halves[0] | (halves[1] << np.uint64(32)))

    def i_v_mad_u32_u24(self, a, pc):
        m24 = np.uint64(0xFFFFFF)
        self._vop3(a, lambda x, y, z: (x & m24) * (y & m24) + z, 3)

    def i_v_lshl_add_u32(self, a, pc):
        self._vop3(a, lambda x, y, z: (x << (y & np.uint64(31))) + z, 3)

    def i_v_min3_u32(self, a, pc):
        self._vop3(a, lambda x, y, z: np.minimum(np.minimum(x, y), z), 3)

    def i_v_min_u32(self, a, pc):
        self._vop2(a, lambda x, y: np.minimum(x, y))

    def i_v_med3_i32(self, a, pc):
        def med3(x, y, z):
            sx, sy, sz = (t.astype(np.uint32).view(np.int32).astype(np.int64) for t in (x, y, z))
            m = np.maximum(np.minimum(sx, sy), np.minimum(np.maximum(sx, sy), sz))
            return (m & 0xFFFFFFFF).astype(np.uint64)
        self._vop3(a, med3, 3)

    def i_s_movk_i32(self, a, pc):
        v = int(a[1], 0) & 0xFFFF
        self.swrite(a[0], (v - 0x10000 if v & 0x8000 else v) & M32)

    def i_v_add3_u32(self, a, pc):
        self._vop3(a, lambda x, y, z: x + y + z, 3)

    def i_v_or3_b32(self, a, pc):
        self._vop3(a, lambda x, y, z: x | y | z, 3)

    def i_v_bfi_b32(self, a, pc):
        self._vop3(a, lambda m, x, y: (m & x) | (~m & y), 3)

    def i_v_bfe_u32(self, a, pc):
        self._vop3(a, lambda x, o, w: (x >> (o & np.uint64(31))) &
                   ((np.uint64(1) << (w & np.uint64(31))) - np.uint64(1)), 3)

    def i_v_alignbit_b32(self, a, pc):
        self._vop3(a, lambda hi, lo, s: (((hi << np.uint64(32)) | lo) >> (s & np.uint64(31))), 3)

    def i_v_lshlrev_b64(self, a, pc):
        s = self.vread(a[1], "SRC0")
        x = self.vread(a[2], "SRC1", 64)
        self.vwrite(a[0], (x << (s & np.uint64(63))) & np.uint64(M64))

    def i_v_bfrev_b32(self, a, pc):
        x = self.vread(a[1], "SRC0").astype(np.uint32)
        r = np.zeros_like(x)
        for k in range(32):
            r |= ((x >> np.uint32(k)) & np.uint32(1)) << np.uint32(31 - k)
        self.vwrite(a[0], r.astype(np.uint64))

    def i_v_mul_u32_u24(self, a, pc):
        m24 = np.uint64(0xFFFFFF)
        self._vop2(a, lambda x, y: (x & m24) * (y & m24))

    def i_v_lshrrev_b64(self, a, pc):
        s = self.vread(a[1], "SRC0")
        x = self.vread(a[2], "SRC1", 64)
        self.vwrite(a[0], x >> (s & np.uint64(63)))

    def _carry_in(self, op):
        return self.lanes_mask(op).astype(np.uint64)

    def i_v_add_co_u32(self, a, pc):
        x, y = self.vread(a[2], "SRC0"), self.vread(a[3], "SRC1")
        r = x + y
        self.wr_lanes(a[1], (r >> np.uint64(32)) != 0)
        self.vwrite(a[0], r & np.uint64(M32))

    def i_v_addc_co_u32(self, a, pc):
        x, y = self.vread(a[2], "SRC0"), self.vread(a[3], "SRC1")
        r = x + y + self._carry_in(a[4])
        self.wr_lanes(a[1], (r >> np.uint64(32)) != 0)
        self.vwrite(a[0], r & np.uint64(M32))

    def i_v_sub_co_u32(self, a, pc):
        x, y = self.vread(a[2], "SRC0"), self.vread(a[3], "SRC1")
        self.wr_lanes(a[1], x < y)
        self.vwrite(a[0], (x - y) & np.uint64(M32))

    def i_v_subb_co_u32(self, a, pc):
        x, y = self.vread(a[2], "SRC0"), self.vread(a[3], "SRC1")
        c = self._carry_in(a[4])
        self.wr_lanes(a[1], x < y + c)
        self.vwrite(a[0], (x - y - c) & np.uint64(M32))

    def i_v_subrev_co_u32(self, a, pc):
        x, y = self.vread(a[2], "SRC0"), self.vread(a[3], "SRC1")
        self.wr_lanes(a[1], y < x)
        self.vwrite(a[0], (y - x) & np.uint64(M32))

    def i_v_subbrev_co_u32(self, a, pc):
        x, y = self.vread(a[2], "SRC0"), self.vread(a[3], "SRC1")
        c = self._carry_in(a[4])
        self.wr_lanes(a[1], y < x + c)
        self.vwrite(a[0], (y - x - c) & np.uint64(M32))

    def i_v_mad_u64_u32(self, a, pc):
        x, y = self.vread(a[2], "SRC0"), self.vread(a[3], "SRC1")
        c = self.vread(a[4], "SRC2", 64)
        r = [int(p) * int(q) + int(t) for p, q, t in zip(x, y, c)]
        self.wr_lanes(a[1], np.array([t >> 64 for t in r], dtype=bool))
        self.vwrite(a[0], np.array([t & M64 for t in r], dtype=np.uint64))

    def _cmp(self, a, f, width=32, signed=False):
        x = self.vread(a[1], "SRC0", width)
        y = self.vread(a[2], "SRC1", width)
        if signed:
            x = x.astype(np.uint32).view(np.int32).astype(np.int64)
            y = y.astype(np.uint32).view(np.int32).astype(np.int64)
        self.wr_lanes(a[0], f(x, y))

    def i_v_cmp_eq_u32(self, a, pc):
        self._cmp(a, lambda x, y: x == y)

    def i_v_cmp_ne_u32(self, a, pc):
        self._cmp(a, lambda x, y: x != y)

    def i_v_cmp_ge_u32(self, a, pc):
        self._cmp(a, lambda x, y: x >= y)

    def i_v_cmp_gt_u32(self, a, pc):
        self._cmp(a, lambda x, y: x > y)

    def i_v_cmp_le_u32(self, a, pc):
        self._cmp(a, lambda x, y: x <= y)

    def i_v_cmp_lt_u32(self, a, pc):
        self._cmp(a, lambda x, y: x < y)

    def i_v_cmp_gt_i32(self, a, pc):
        self._cmp(a, lambda x, y: x > y, signed=True)

    def i_v_cmp_eq_u64(self, a, pc):
        self._cmp(a, lambda x, y: x == y, width=64)

    def i_v_cmp_lt_u64(self, a, pc):
        self._cmp(a, lambda x, y: x < y, width=64)

    def i_v_cmp_gt_u64(self, a, pc):
        self._cmp(a, lambda x, y: x > y, width=64)

    def i_v_cmp_ge_u64(self, a, pc):
        self._cmp(a, lambda x, y: x >= y, width=64)

    def i_v_cndmask_b32(self, a, pc):
        x, y = self.vread(a[1], "SRC0"), self.vread(a[2], "SRC1")
        m = self.lanes_mask(a[3])
        self.vwrite(a[0], np.where(m, y, x))

    # ---- f64 (the division reciprocal) ----
    @staticmethod
    def _f(u):
        return np.asarray(u, dtype=np.uint64).view(np.float64)

    @staticmethod
    def _u(f):
        return np.asarray(f, dtype=np.float64).view(np.uint64)

    def i_v_cvt_f64_u32(self, a, pc):
        x = self.vread(a[1], "SRC0")
        self.vwrite(a[0], self._u(x.astype(np.float64)))

    def i_v_rcp_f64(self, a, pc):
        x = self._f(self.vread(a[1], "SRC0", 64))
        with np.errstate(divide="ignore"):
            r = 1.0 / x
        if self.rcp_noise:
            r = r * (1.0 + self.rng.uniform(-self.rcp_noise, self.rcp_noise, NL))
        self.vwrite(a[0], self._u(r))

    def i_v_fma_f64(self, a, pc):
        x = self._f(self.vread(a[1], "SRC0", 64))
        y = self._f(self.vread(a[2], "SRC1", 64))
        z = self._f(self.vread(a[3], "SRC2", 64))
        # fused: evaluate exactly with Python fractions-free long double path
        r = np.array([float(np.longdouble(p) * np.longdouble(q) + np.longdouble(t))
                      for p, q, t in zip(x, y, z)])
        self.vwrite(a[0], self._u(r))

    def i_v_ldexp_f64(self, a, pc):
        x = self._f(self.vread(a[1], "SRC0", 64))
        e = self.vread(a[2], "SRC1").astype(np.int64)
        self.vwrite(a[0], self._u(np.ldexp(x, e)))

    def i_v_add_f64(self, a, pc):
        x = self._f(self.vread(a[1], "SRC0", 64))
        y = self._f(self.vread(a[2], "SRC1", 64))
        self.vwrite(a[0], self._u(x + y))

    def i_v_cvt_u32_f64(self, a, pc):
        x = self._f(self.vread(a[1], "SRC0", 64))
        r = np.where(np.isnan(x), 0, np.clip(np.trunc(x), 0, M32)).astype(np.uint64)
        self.vwrite(a[0], r)

    # ---------------- memory ----------------
    def _soff(self, tok: str) -> int:
        m = re.fullmatch(r"offset:(\d+)", tok)
        return int(m.group(1)) if m else 0

    def i_global_load_dword(self, a, pc):
        self._gload(a, 1)

    def i_global_load_dwordx4(self, a, pc):
        self._gload(a, 4)

    def _gaddr(self, voff: str, sbase: str, extra: List[str]):
        base = self.sread(sbase, 64)
        off = self._soff(extra[0]) if extra else 0
        vo = self.vread(voff, valu=False)
        return [(base + int(vo[l]) + off) & M64 for l in range(NL)]

    def _gload(self, a, n):
        dst, cnt = self.vidx(a[0], None, False)
        if cnt != n:
            raise SimError("load width mismatch")
        addrs = self._gaddr(a[1], a[2], a[3:])
        act = self._act()
        vals = [[self.mem.read32(addrs[l] + 4 * i) if act[l] else 0 for l in range(NL)]
                for i in range(n)]
        for i in range(n):
            def apply(i=i):
                self.v[dst + i] = np.where(act, np.array(vals[i], dtype=np.uint64), self.v[dst + i])
            self._defer("vm", ("v", dst + i), apply, lanes=act.copy())

    def i_global_store_dword(self, a, pc):
        addrs = self._gaddr(a[0], a[2], a[3:])
        data = self.vread(a[1], valu=False)
        act = self._act()
        for l in range(NL):
            if act[l]:
                self.mem.write32(addrs[l], int(data[l]))

    def _scratch_store(self, a, n):
        if a[0] != "off":
            raise SimError("scratch: vaddr form not modelled")
        src, _ = self.vidx(a[1], None, False)
        off = self.sread(a[2]) + (self._soff(a[3]) if len(a) > 3 else 0)
        act = self._act()
        for l in range(NL):
            if act[l]:
                if off + 4 * n > len(self.scratch[l]):
                    raise SimError("scratch out of bounds")
                for i in range(n):
                    self._check(("v", src + i))
                    struct.pack_into("<I", self.scratch[l], off + 4 * i, int(self.v[src + i][l]))

    def _scratch_load(self, a, n):
        dst, _ = self.vidx(a[0], None, False)
        if a[1] != "off":
            raise SimError("scratch: vaddr form not modelled")
        off = self.sread(a[2]) + (self._soff(a[3]) if len(a) > 3 else 0)
        act = self._act()
        vals = [[struct.unpack_from("<I", self.scratch[l], off + 4 * i)[0] for l in range(NL)]
                for i in range(n)]
        for i in range(n):
            def apply(i=i):
                self.v[dst + i] = np.where(act, np.array(vals[i], dtype=np.uint64), self.v[dst + i])
            self._defer("vm", ("v", dst + i), apply)

    def i_scratch_store_dwordx4(self, a, pc):
        self._scratch_store(a, 4)

    def i_scratch_store_dword(self, a, pc):
        self._scratch_store(a, 1)

    def i_scratch_load_dwordx4(self, a, pc):
        self._scratch_load(a, 4)

    def i_scratch_load_dword(self, a, pc):
        self._scratch_load(a, 1)

    def i_ds_write_b128(self, a, pc):
        addr = self.vread(a[0], valu=False)
        src, _ = self.vidx(a[1], None, False)
        off = self._soff(a[2]) if len(a) > 2 else 0
        act = self._act()
        for l in range(NL):
            if act[l]:
                for i in range(4):
                    self._check(("v", src + i))
                    struct.pack_into("<I", self.lds, int(addr[l]) + off + 4 * i, int(self.v[src + i][l]))

    def i_ds_write_b32(self, a, pc):
        addr = self.vread(a[0], valu=False)
        src, _ = self.vidx(a[1], None, False)
        off = self._soff(a[2]) if len(a) > 2 else 0
        act = self._act()
        self._check(("v", src))
        for l in range(NL):
            if act[l]:
                struct.pack_into("<I", self.lds, int(addr[l]) + off, int(self.v[src][l]))

    def i_ds_read_b32(self, a, pc):
        dst, _ = self.vidx(a[0], None, False)
        addr = self.vread(a[1], valu=False)
        off = self._soff(a[2]) if len(a) > 2 else 0
        act = self._act()
        vals = [struct.unpack_from("<I", self.lds, int(addr[l]) + off)[0] for l in range(NL)]

        def apply():
            self.v[dst] = np.where(act, np.array(vals, dtype=np.uint64), self.v[dst])
        self._defer("lgkm", ("v", dst), apply)

    def i_ds_read_b128(self, a, pc):
        dst, _ = self.vidx(a[0], None, False)
        addr = self.vread(a[1], valu=False)
        off = self._soff(a[2]) if len(a) > 2 else 0
        act = self._act()
        vals = [[struct.unpack_from("<I", self.lds, int(addr[l]) + off + 4 * i)[0] for l in range(NL)]
                for i in range(4)]
        for i in range(4):
            def apply(i=i):
                self.v[dst + i] = np.where(act, np.array(vals[i], dtype=np.uint64), self.v[dst + i])
            self._defer("lgkm", ("v", dst + i), apply)


# ---------------------------------------------------------------------------
# driving the interpreter body like mg_interp_asm does
# ---------------------------------------------------------------------------

def _operands():
    """inline-asm operands -> the registers the kernel pins them to
    (asmgen.PINNED): the simulator runs the exact text, compiled programs
    (mythril_amd/jit.py) included."""
    from mythril_amd import asmgen
    return {"%%[%s]" % k: r for k, r in asmgen.PINNED.items()}


OPERANDS = _operands()


def _set_input(w, name: str, val: int):
    """Write a kernel input into its pinned register(s)."""
    from mythril_amd import asmgen
    reg = asmgen.PINNED[name]
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", reg) or re.fullmatch(r"s(\d+)", reg)
    base = int(m.group(1))
    w.s[base] = val & M32
    if "[" in reg:
        w.s[base + 1] = (val >> 32) & M32


def _vreg_of(name: str) -> int:
    from mythril_amd import asmgen
    return int(asmgen.PINNED[name][1:])


def handler_table(lines: List[str], n_handlers: int) -> List[int]:
    """Run the body in query mode (as mg_init does) and return the table."""
    mem = Memory()
    desc = mem.alloc(bytes(80), "desc")
    table = mem.alloc(bytes(4 * n_handlers), "table")
    w = Wave(lines, OPERANDS, mem)
    _set_input(w, "desc", desc)
    _set_input(w, "mode", 2)
    _set_input(w, "table", table)
    w.run()
    buf = mem.region(table)
    return list(struct.unpack_from("<%dI" % n_handlers, buf, 0))


_CACHE: Dict[str, object] = {}


def body_and_table():
    """(asm lines, handler offset table) of the current generator."""
    if "lines" not in _CACHE:
        from mythril_amd import asmgen
        lines = asmgen.generate()
        _CACHE["lines"] = lines
        _CACHE["table"] = handler_table(lines, asmgen.NUM_HANDLERS)
    return _CACHE["lines"], _CACHE["table"]


def translate(prog, n_lds: int):
    """Records + translator masks through the library's host-only mg_translate."""
    import ctypes as C
    from mythril_amd.asmgen import NUM_HANDLERS
    from mythril_amd.engine import load_library
    lib = load_library(check_digest=False)     # host-only translator
    _, table = body_and_table()
    code = np.ascontiguousarray(prog.code, dtype=np.uint32)
    tab = np.array(table, dtype=np.uint32)
    rec = np.zeros((2 * prog.n_ins + 3) * 8, dtype=np.uint32)
    masks = np.zeros(8 * 4096, dtype=np.uint32)
    nr, nm = C.c_uint32(0), C.c_uint32(0)
    from mythril_amd import asmgen
    if prog.nreg != asmgen.NREG:
        raise SimError("a %d-slot program; this process simulates the %d-slot interpreter "
                       "(MYTHGPU_NREG)" % (prog.nreg, asmgen.NREG))
    rc = lib.mg_translate(code.ctypes.data_as(C.c_void_p), prog.n_ins, prog.consts.shape[0], n_lds,
                          prog.nreg, tab.ctypes.data_as(C.c_void_p), NUM_HANDLERS,
                          rec.ctypes.data_as(C.c_void_p), rec.size, C.byref(nr),
                          masks.ctypes.data_as(C.c_void_p), masks.size, C.byref(nm))
    if rc != 0:
        raise SimError("mg_translate failed: %d" % rc)
    return rec[:nr.value], masks[:nm.value]


GOLD = 0x9E3779B97F4A7C15


def _limbs(v: int) -> list:
    return [(v >> (32 * j)) & M32 for j in range(8)]


def boundary_table() -> np.ndarray:
    """The generator's boundary table as mg_api.cpp builds it: entry
    kind * 256 + p = 0, 1, 1 << p, 2^256 - 1, (1 << p) + 1, (1 << p) - 1."""
    t = np.zeros((6, 256, 8), dtype=np.uint32)
    for p in range(256):
        for kind, val in enumerate((0, 1, 1 << p, (1 << 256) - 1, (1 << p) + 1, (1 << p) - 1)):
            t[kind, p] = _limbs(val)
    return t


def expanded_pool(consts: np.ndarray) -> np.ndarray:
    """(v - 1, v, v + 1) mod 2^256 for every constant (mg_load_program)."""
    out = np.zeros((consts.shape[0], 3, 8), dtype=np.uint32)
    for c in range(consts.shape[0]):
        v = sum(int(consts[c, j]) << (32 * j) for j in range(8))
        for d in range(3):
            out[c, d] = _limbs((v + d - 1) % (1 << 256))
    return out


def simulate(prog, soa: Optional[np.ndarray] = None, gen=None, n_lds: int = 6,
             active: int = (1 << NL) - 1, rcp_noise: float = 0.0, want_leaves: bool = False,
             jit: bool = False):
    """Run one 64-lane wave of the assembly interpreter on a compiled
    Program.  Eval mode: soa [n_leaves][8][64] u32.  Generator mode: gen =
    (seed, prog_seed, first_index, leafgens) with leafgens the engine's
    LeafGen list.  ``jit``: the program's compiled code (mythril_amd/jit.py)
    is appended and entered through the descriptor's jit_entry, as on the
    GPU.  Returns (root bits [64] bool, probes [n_probes][8][64],
    leaves_out [n_leaves][8][64] or None, wave)."""
    lines, _ = body_and_table()
    if jit:
        from mythril_amd import jit as J
        from mythril_amd.engine import default_leafgen
        lg = gen[3] if gen is not None else default_leafgen(prog)
        ps = gen[1] if gen is not None else 0
        lines = list(lines) + ["    s_endpgm"] + J.program_asm(prog, lg, ps, ".Ljp0", n_lds) + \
            J.bodies()
    rec, masks = translate(prog, n_lds)
    mem = Memory()
    pc = np.ascontiguousarray(prog.consts, dtype=np.uint32).reshape(-1, 8)
    consts = np.concatenate([pc.reshape(-1), masks, expanded_pool(pc).reshape(-1)]).astype(np.uint32)
    pool_base = pc.shape[0] + len(masks) // 8         # expanded pool, in 32-byte entries
    c_base = mem.alloc(consts.tobytes(), "consts")
    x_base = mem.alloc(rec.astype(np.uint32).tobytes(), "records")
    n_leaves = len(prog.leaves)
    gdev = np.zeros((max(1, n_leaves), 8), dtype=np.uint32)
    seed = prog_seed = first = 0
    if gen is not None:
        seed, prog_seed, first, leafgens = gen
        for i, g in enumerate(leafgens):
            salt = ((prog_seed * 0xD1B54A32D192ED03) ^ ((i + 1) * 0x8CB92BA72F3D8DD7)) & M64
            gdev[i] = [g.width, (pool_base + 3 * g.pool_off) * 32, g.pool_n, g.pct_uniform,
                       g.pct_small, g.pct_boundary, salt & M32, salt >> 32]
        # LEAFD records carry the generator parameters (mg_load_program)
        from mythril_amd import asmgen
        _, table = body_and_table()
        leafd = {table[asmgen.hid(asmgen.AOP["LEAFD"], var | w, bank)]
                 for var in range(asmgen.NREG) for w in (0, asmgen.V_WAITD) for bank in (0, 1)}
        rec = rec.copy()
        for r in range(0, len(rec) - 7, 8):
            li = int(rec[r + 4])
            if int(rec[r]) in leafd and li < n_leaves:
                g = gdev[li]
                rec[r + 1], rec[r + 2], rec[r + 3], rec[r + 5] = g[1], g[6], g[7], g[2]
                rec[r + 7] = int(g[3]) | int(g[4]) << 8 | int(g[5]) << 16
        x_base = mem.alloc(rec.astype(np.uint32).tobytes(), "records")
    g_base = mem.alloc(gdev.tobytes(), "gen")
    b_base = mem.alloc(boundary_table().tobytes(), "btab")
    w = Wave(lines, OPERANDS, mem, rcp_noise=rcp_noise)
    jit_entry = w.addr_of(".Ljp0") if jit else 0
    desc = struct.pack("<QQQIIIIQQQQ", 0, c_base, g_base, prog.n_ins, n_leaves, 0, 0,
                       prog_seed & M64, x_base, b_base, jit_entry)
    d_base = mem.alloc(desc, "desc")
    lv = soa if soa is not None else np.zeros((max(1, n_leaves), 8, NL), dtype=np.uint32)
    l_base = mem.alloc(np.ascontiguousarray(lv, dtype=np.uint32).tobytes(), "leaves")
    n_pr = max(1, prog.n_probes)
    p_base = mem.alloc(bytes(n_pr * 8 * NL * 4), "probes")
    o_base = mem.alloc(bytes(max(1, n_leaves) * 8 * NL * 4), "leaves_out") if want_leaves else 0
    for name, val in (("desc", d_base), ("seed", seed & M64), ("first", first & M64),
                      ("leaves", l_base), ("stride", NL), ("lout", o_base),
                      ("probes", p_base if prog.n_probes else 0), ("active", active),
                      ("mode", 1 if gen is not None else 0), ("scr", 0)):
        _set_input(w, name, val)
    idx = [(first + lane) & M64 for lane in range(NL)]      # the shell's first + lane
    w.v[_vreg_of("idx_lo")] = np.array([i & M32 for i in idx], dtype=np.uint64)
    w.v[_vreg_of("idx_hi")] = np.array([i >> 32 for i in idx], dtype=np.uint64)
    w.v[_vreg_of("lds")] = np.arange(NL, dtype=np.uint64) * 16
    w.run(max_steps=20_000_000)
    if w.pending:
        raise SimError("loads still pending at exit: %s" % sorted(w.pending))
    root = (w.v[_vreg_of("root")] & 1).astype(bool)
    probes = np.frombuffer(bytes(mem.region(p_base)), dtype=np.uint32).reshape(n_pr, 8, NL)
    lout = None
    if want_leaves:
        lout = np.frombuffer(bytes(mem.region(o_base)), dtype=np.uint32).reshape(-1, 8, NL)
    return root, probes, lout, w
