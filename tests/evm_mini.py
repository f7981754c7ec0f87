"""Test infrastructure: lower a straight-line VMTest program into the DAGs
LASER would hand to ``get_model``.

Each PUSH becomes a fresh 256-bit *variable* ``p<i>`` whose value goes into
the assignment, so a (DAG, assignment) pair is a real evaluation problem for
the engine and not a folded constant.  Opcode lowering follows
``mythril/laser/ethereum/instructions.py`` (file:line per opcode below),
including the places where LASER inspects a concrete value (division by a
concrete zero → 0, ``BYTE`` with a concrete index, ``SIGNEXTEND`` with a
concrete byte count); those decisions use the value of the operand under the
assignment, which is what ``simplify`` would have produced on the concrete
program.
"""

from mythril_amd.smt import (BitVec, Bool, Concat, Extract, If, LShR, Not, SRem, UDiv, UGT,
                             ULT, URem, symbol_factory)

TT256 = 1 << 256
TT256M1 = TT256 - 1


def _bv(x) -> BitVec:
    """``util.pop_bitvec`` (``laser/ethereum/util.py:67-88``)."""
    if isinstance(x, Bool):
        return If(x, symbol_factory.BitVecVal(1, 256), symbol_factory.BitVecVal(0, 256))
    if isinstance(x, int):
        return symbol_factory.BitVecVal(x, 256)
    return x


def lower_program(code_hex: str, evaluate):
    """Return (assignment_vars, stores, divergent).  ``stores`` lists
    (key expression, value expression) per SSTORE; ``evaluate(expr, vars)``
    must return the value of ``expr`` under the variables pushed so far.  ``divergent``
    is True when the program hits a case where LASER's ADDMOD/MULMOD lowering
    (``instructions.py:580,595``: 256-bit ``URem(URem(a,n)+URem(b,n),n)``)
    differs from EVM semantics: the inner sum/product overflows 2^256, or the
    modulus is 0 (EVM gives 0, ``bvurem x 0 = x``)."""
    code = bytes.fromhex(code_hex)
    stack = []
    vars_ = {}
    stores = []
    divergent = [False]
    i = 0

    def concrete(e):
        return evaluate(e, vars_)

    def push_var(v):
        name = "p%d" % len(vars_)
        vars_[name] = v
        stack.append(symbol_factory.BitVecSym(name, 256))

    while i < len(code):
        op = code[i]
        i += 1
        if 0x60 <= op <= 0x7F:
            n = op - 0x5F
            push_var(int.from_bytes(code[i:i + n].ljust(n, b"\0"), "big"))
            i += n
            continue
        if 0x80 <= op <= 0x8F:
            stack.append(stack[-(op - 0x7F)])
            continue
        if 0x90 <= op <= 0x9F:
            k = op - 0x8E
            stack[-1], stack[-k] = stack[-k], stack[-1]
            continue
        if op == 0x00:
            break
        if op == 0x50:
            stack.pop()
        elif op == 0x01:                      # add_ :434
            stack.append(_bv(stack.pop()) + _bv(stack.pop()))
        elif op == 0x02:                      # mul_ :466
            stack.append(_bv(stack.pop()) * _bv(stack.pop()))
        elif op == 0x03:                      # sub_ :450
            stack.append(_bv(stack.pop()) - _bv(stack.pop()))
        elif op in (0x04, 0x05, 0x06, 0x07):  # div_/sdiv_/mod_/smod_ :482-567
            s0, s1 = _bv(stack.pop()), _bv(stack.pop())
            if concrete(s1) == 0:
                stack.append(symbol_factory.BitVecVal(0, 256))
            elif op == 0x04:
                stack.append(UDiv(s0, s1))
            elif op == 0x05:
                stack.append(s0 / s1)
            elif op == 0x06:
                stack.append(URem(s0, s1))
            else:
                stack.append(SRem(s0, s1))
        elif op in (0x08, 0x09):              # addmod_/mulmod_ :570-597
            s0, s1, s2 = _bv(stack.pop()), _bv(stack.pop()), _bv(stack.pop())
            a, b, n = concrete(s0), concrete(s1), concrete(s2)
            if n == 0 or ((a % n + b % n) if op == 0x08 else (a % n) * (b % n)) >= TT256:
                divergent[0] = True
            if op == 0x08:
                stack.append(URem(URem(s0, s2) + URem(s1, s2), s2))
            else:
                stack.append(URem(URem(s0, s2) * URem(s1, s2), s2))
        elif op == 0x0B:                      # signextend_ :634-662
            s0, s1 = stack.pop(), _bv(stack.pop())
            k = concrete(_bv(s0))
            if k <= 31:
                testbit = k * 8 + 7
                if concrete(s1) & (1 << testbit):
                    stack.append(s1 | (TT256 - (1 << testbit)))
                else:
                    stack.append(s1 & ((1 << testbit) - 1))
            else:
                stack.append(s1)
        elif op == 0x10:                      # lt_ :666
            stack.append(ULT(_bv(stack.pop()), _bv(stack.pop())))
        elif op == 0x11:                      # gt_ :678
            stack.append(UGT(_bv(stack.pop()), _bv(stack.pop())))
        elif op == 0x12:                      # slt_ :692
            stack.append(_bv(stack.pop()) < _bv(stack.pop()))
        elif op == 0x13:                      # sgt_ :704
            stack.append(_bv(stack.pop()) > _bv(stack.pop()))
        elif op == 0x14:                      # eq_ :717
            a, b = _bv(stack.pop()), _bv(stack.pop())
            stack.append(a == b)
        elif op == 0x15:                      # iszero_ :745
            v = stack.pop()
            e = Not(v) if isinstance(v, Bool) else v == 0
            stack.append(If(e, symbol_factory.BitVecVal(1, 256), symbol_factory.BitVecVal(0, 256)))
        elif op in (0x16, 0x17):              # and_/or_ :330-376
            a, b = _bv(stack.pop()), _bv(stack.pop())
            stack.append(a & b if op == 0x16 else a | b)
        elif op == 0x18:                      # xor_ :379
            stack.append(_bv(stack.pop()) ^ _bv(stack.pop()))
        elif op == 0x19:                      # not_ :390
            stack.append(symbol_factory.BitVecVal(TT256M1, 256) - _bv(stack.pop()))
        elif op == 0x1A:                      # byte_ :401-430
            op0, op1 = stack.pop(), _bv(stack.pop())
            index = concrete(_bv(op0))
            offset = (31 - index) * 8 if index < 2 ** 64 else -1
            if offset >= 0:
                stack.append(Concat(symbol_factory.BitVecVal(0, 248), Extract(offset + 7, offset, op1)))
            else:
                stack.append(symbol_factory.BitVecVal(0, 256))
        elif op == 0x1B:                      # shl_ :526
            shift, value = _bv(stack.pop()), _bv(stack.pop())
            stack.append(value << shift)
        elif op == 0x1C:                      # shr_ :534
            shift, value = _bv(stack.pop()), _bv(stack.pop())
            stack.append(LShR(value, shift))
        elif op == 0x1D:                      # sar_ :542
            shift, value = _bv(stack.pop()), _bv(stack.pop())
            stack.append(value >> shift)
        elif op == 0x55:                      # sstore_ :1492
            index, value = _bv(stack.pop()), _bv(stack.pop())
            stores.append((index, value))
        else:
            raise NotImplementedError(hex(op))
    return vars_, stores, divergent[0]

