"""The C-ABI library loads without a GPU and exports every function that
include/mythgpu.h declares (no compute calls here)."""

import ctypes
import os
import re

from mythril_amd import build
from mythril_amd.engine import EXPORTS, load_library

HDR = os.path.join(build.ROOT, "include", "mythgpu.h")


def declared():
    text = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|float|const char\*)\s+(mg_\w+)\s*\(", text, re.M)))


def test_library_built_from_current_generator():
    from mythril_amd import asmgen
    assert load_library().mg_asm_digest().decode() == asmgen.digest()


def test_library_exports_every_declared_symbol():
    lib = load_library()
    names = declared()
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(EXPORTS)
    cfg = (ctypes.c_uint32 * 4)()
    assert lib.mg_config(cfg, 4) == 0 and cfg[1] >= 8


def test_version_without_gpu():
    assert load_library().mg_version() == 3


def test_ir_header_matches_python_table():
    from mythril_amd import irdefs
    assert irdefs.NUM_OPS == 37 and irdefs.ROOT == 32 and irdefs.CDWX == 36 and irdefs.TRASH == irdefs.NREG - 1
