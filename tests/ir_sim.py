"""Test infrastructure: a reference executor for compiled mythgpu IR.

Executes a :class:`mythril_amd.ir.Program` instruction by instruction on
Python integers, with the op semantics taken from the oracle
(``oracle/smtlib_ref.py``).  Running it against direct oracle evaluation of
the source DAG checks the host compiler (lowering, scheduling, register
allocation, spilling) on the CPU; the GPU tests then check the kernel against
the same oracle.
"""

from mythril_amd import irdefs as I
from oracle import smtlib_ref as R


def _signed(x, w):
    return x - (1 << w) if x >> (w - 1) else x


def run(program, leaf_vals):
    regs = [0] * I.NREG
    spill = {}
    root = 1
    probes = {}
    consts = program.const_values
    for row in program.code:
        w0, w1, imm = int(row[0]), int(row[1]), int(row[2])
        op, w = w0 & 0xFF, (w0 >> 8) & 0x3FF
        d, a, b, c = w1 & 0xFF, (w1 >> 8) & 0xFF, (w1 >> 16) & 0xFF, (w1 >> 24) & 0xFF
        x, y = regs[a], regs[b]
        m = (1 << w) - 1 if w else 0
        r = 0
        if op == I.CONST:
            r = consts[imm]
        elif op == I.LEAF:
            r = leaf_vals[imm] & m
        elif op == I.SPILL:
            spill[imm] = x
        elif op == I.RELOAD:
            r = spill[imm]
        elif op == I.ADD:
            r = (x + y) & m
        elif op == I.SUB:
            r = (x - y) & m
        elif op == I.NEG:
            r = (-x) & m
        elif op == I.MUL:
            r = (x * y) & m
        elif op == I.UDIV:
            r = R.bvudiv(x, y, w)
        elif op == I.UREM:
            r = R.bvurem(x, y, w)
        elif op == I.SDIV:
            r = R.bvsdiv(x, y, w)
        elif op == I.SREM:
            r = R.bvsrem(x, y, w)
        elif op == I.SMOD:
            r = R.bvsmod(x, y, w)
        elif op == I.AND:
            r = x & y
        elif op == I.OR:
            r = x | y
        elif op == I.XOR:
            r = x ^ y
        elif op == I.NOT:
            r = ~x & m
        elif op == I.SHL:
            r = R.bvshl(x, y, w)
        elif op == I.LSHR:
            r = R.bvlshr(x, y, w)
        elif op == I.ASHR:
            r = R.bvashr(x, y, w)
        elif op == I.EQ:
            r = int(x == y)
        elif op == I.ULT:
            r = int(x < y)
        elif op == I.ULE:
            r = int(x <= y)
        elif op == I.SLT:
            r = int(_signed(x, w) < _signed(y, w))
        elif op == I.SLE:
            r = int(_signed(x, w) <= _signed(y, w))
        elif op == I.UMULNO:
            r = int(x * y < (1 << w))
        elif op == I.ITE:
            r = x if regs[c] & 1 else y
        elif op == I.CONCAT:
            r = ((x << imm) | y) & m
        elif op == I.EXTRACT:
            r = (x >> imm) & m
        elif op == I.SEXT:
            r = _signed(x, imm) & m
        elif op == I.OUT:
            probes[imm] = x
        elif op == I.ROOT:
            root &= x & 1
        elif op == I.NOP:
            pass
        elif op == I.MOV:
            r = x
        elif op == I.BCAST:
            r = (x & 0xFF) * int("01" * 32, 16)
        elif op == I.CDWE:
            r = x
            if y < 32:
                sh = 8 * (31 - y)
                r = (x & ~(0xFF << sh)) | ((regs[c] & 0xFF) << sh)
        elif op == I.CDWX:
            r = x
            for i in range(32):
                if not _signed((y + i) % (1 << 256), 256) < _signed(regs[c], 256):
                    r &= ~(0xFF << (8 * (31 - i)))
        else:
            raise AssertionError("op %d" % op)
        if w0 & I.ROOT_FLAG:
            root &= r & 1
        if op in (I.ITE, I.AND, I.OR, I.XOR, I.MOV, I.CONST):
            # the IR contract: a value is canonical at its instruction's width
            # (the kernel picks one-limb / masked handlers from it)
            assert r >> w == 0, "op %d writes a %d-bit value at width %d" % (op, r.bit_length(), w)
        if op not in (I.SPILL, I.OUT, I.ROOT, I.NOP):   # these write no slot (mg_host.cpp)
            regs[d] = r
    return root, [probes.get(i, 0) for i in range(program.n_probes)]
