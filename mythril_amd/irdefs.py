"""Opcode table of the mythgpu IR, read from ``include/mythgpu_ir.h`` so the
Python compiler and the HIP interpreter can never disagree."""

import os
import re

_HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                    "mythgpu_ir.h")


def _parse():
    ops, defs = {}, {}
    with open(_HDR) as fh:
        text = fh.read()
    # opcodes: the enum mg_op body only (comments elsewhere may read "MG_X = n")
    body = text[text.index("enum mg_op"):]
    body = body[:body.index("};")]
    for m in re.finditer(r"\bMG_([A-Z0-9_]+)\s*=\s*(\d+)\s*[,\n]", body):
        ops[m.group(1)] = int(m.group(2))
    for m in re.finditer(r"#define\s+MG_([A-Z_]+)\s+(\d+)", text):
        defs[m.group(1)] = int(m.group(2))
    return ops, defs


OPS, DEFINES = _parse()
NREG = int(os.environ.get("MYTHGPU_NREG", DEFINES["NREG"]))   # (A/B builds: asmgen.NREG)
TRASH = NREG - 1
MAX_WIDTH = DEFINES["MAX_WIDTH"]
MAX_LDS = DEFINES["MAX_LDS"]
MAX_LDS_DS = DEFINES["MAX_LDS_DS"]


def check_lds_slots(n) -> int:
    """LDS spill regions a context / compiled program may use: 0 ..
    MG_MAX_LDS_DS (compiled programs address every LDS half with a DS
    instruction's 16-bit offset; more regions would assemble to an image
    the assembler refuses).  Raises ValueError."""
    try:
        v = int(n)
    except (TypeError, ValueError):
        raise ValueError("LDS spill regions %r: not an integer" % (n,)) from None
    if not 0 <= v <= MAX_LDS_DS:
        raise ValueError("LDS spill regions %d: the DS offsets of compiled programs reach "
                         "%d regions at most (MG_MAX_LDS_DS)" % (v, MAX_LDS_DS))
    return v
ROOT_FLAG = 1 << 18          # MG_ROOT_FLAG: w0 bit 18, ROOT fused into the producer
MAX_PSLOTS = DEFINES["MAX_PSLOTS"]
NUM_OPS = OPS["NUM_OPS"]
OPNAME = {v: k for k, v in OPS.items() if k != "NUM_OPS"}

globals().update({k: v for k, v in OPS.items()})


def w0(op: int, width: int) -> int:
    return op | (width << 8)


def w1(d: int, a: int = 0, b: int = 0, c: int = 0) -> int:
    return d | (a << 8) | (b << 16) | (c << 24)
