"""The C-ABI library loads without a GPU and exports every function that
include/mythgpu.h declares (no compute calls here)."""

import ctypes
import os
import re

import pytest

from mythril_amd import build
from mythril_amd.engine import EXPORTS, load_library

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

HDR = os.path.join(build.ROOT, "include", "mythgpu.h")


def declared():
    text = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|float|const char\*)\s+(mg_\w+)\s*\(", text, re.M)))


def test_library_built_from_current_generator():
    from mythril_amd import asmgen
    lib = load_library()
    with asmgen.layout(16):
        assert lib.mg_asm_digest().decode() == asmgen.digest()
    for nreg in (16, 11):
        with asmgen.layout(nreg):
            assert lib.mg_asm_digest_layout(nreg).decode() == asmgen.digest()
    assert lib.mg_asm_digest_layout(12) is None


def test_library_exports_every_declared_symbol():
    lib = load_library()
    names = declared()
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(EXPORTS)
    cfg = (ctypes.c_uint32 * 4)()
    assert lib.mg_config(cfg, 4) == 0 and cfg[1] >= 8


def test_one_library_holds_both_register_layouts():
    """one library, both interpreters.  mg_layouts lists
    (16 slots, 3 waves, 6 LDS regions) and (11, 4, 5); the 11-slot body is
    the generator's under that layout (digest, and a 128-VGPR budget: four
    waves per SIMD), and the translator refuses a slot the layout lacks."""
    import numpy as np
    from mythril_amd import asmgen
    from mythril_amd.engine import layouts
    assert layouts() == {16: (3, 6), 11: (4, 5)} == {n: v for n, v in build.LAYOUTS.items()}
    with asmgen.layout(11):
        assert asmgen.NVGPR_KERNEL == 128 and asmgen.YB == 8 + 8 * 11
    assert asmgen.NVGPR_KERNEL == 168 or asmgen.NREG == 11      # restored
    lib = load_library()
    code = np.array([[2 | (8 << 8), 13, 0, 0]], dtype=np.uint32)   # CONST w8 into slot 13
    ident = np.arange(asmgen.NUM_HANDLERS, dtype=np.uint32)
    rec = np.zeros(64, dtype=np.uint32)
    masks = np.zeros(64, dtype=np.uint32)
    nw, nm = ctypes.c_uint32(), ctypes.c_uint32()
    args = (ident.ctypes.data_as(ctypes.c_void_p), asmgen.NUM_HANDLERS,
            rec.ctypes.data_as(ctypes.c_void_p), 64, ctypes.byref(nw),
            masks.ctypes.data_as(ctypes.c_void_p), 64, ctypes.byref(nm))
    c = code.ctypes.data_as(ctypes.c_void_p)
    assert lib.mg_translate(c, 1, 1, 0, 16, *args) == 0
    assert lib.mg_translate(c, 1, 1, 0, 11, *args) != 0       # slot 13 of 11
    assert lib.mg_translate(c, 1, 1, 0, 12, *args) != 0       # no 12-slot layout


def test_version_without_gpu():
    assert load_library().mg_version() == 4


def test_ir_header_matches_python_table():
    from mythril_amd import irdefs
    assert irdefs.NUM_OPS == 37 and irdefs.ROOT == 32 and irdefs.CDWX == 36 and irdefs.TRASH == irdefs.NREG - 1


def test_every_device_entry_point_sets_its_device():
    """every exported entry point that touches device
    memory or launches (HIP calls, launches, device blocks) makes its
    context's device current first, so one host thread may drive contexts
    on different devices.  Source scan of the C ABI (runs without a GPU)."""
    import re
    src = open(os.path.join(build.ROOT, "mythril_amd", "csrc", "mg_api.cpp")).read()
    host_only = {"mg_version", "mg_config", "mg_translate", "mg_asm_digest", "mg_last_error",
                 "mg_last_kernel_ms", "mg_runtime_info", "mg_init", "mg_asm_digest_layout",
                 "mg_layouts"}
    bodies = {}
    for m in re.finditer(r"^(?:int|void|float|const char\*) (mg_\w+)\([^;{]*\)\s*\{", src, re.M):
        depth, i = 1, m.end()
        while depth:
            depth += {"{": 1, "}": -1}.get(src[i], 0)
            i += 1
        bodies[m.group(1)] = src[m.end():i]
    assert {"mg_batch_eval_gen", "mg_batch_search", "mg_load_program", "mg_eval"} <= set(bodies)
    touches = re.compile(r"\bhip[A-Z]\w*\(|\blaunch\(|dev_alloc\(|dev_release\(|workspace\(")
    missing = [f for f, b in bodies.items()
               if f not in host_only and touches.search(b) and "hipSetDevice" not in b]
    assert missing == []
    # mg_init(_layout) selects the device it is given
    assert "hipSetDevice(device)" in bodies["mg_init_layout"]


def test_lds_regions_beyond_ds_offsets_are_refused_when_configured():
    """MYTHGPU_LDS_SLOTS=10 used to yield compiled code the
    assembler rejected (LDS halves past a DS instruction's 16-bit offset).
    Such a region count is refused where it is configured — the compiled-
    program renderer, the context's region count (engine.lds_slots_for, and
    mg_init in the library) — and the
    largest accepted count, MG_MAX_LDS_DS, renders DS offsets that fit."""
    import re
    import subprocess
    import sys
    import bench
    from mythril_amd import irdefs, jit
    from mythril_amd.engine import default_leafgen
    assert irdefs.MAX_LDS_DS == 8
    assert irdefs.check_lds_slots("8") == 8 and irdefs.check_lds_slots(0) == 0
    for bad in (9, 10, -1, "x", None):
        with pytest.raises(ValueError):
            irdefs.check_lds_slots(bad)
    _, prog, _, _ = bench.compile_unit(("c3", 16))           # a spill-heavy unit
    with pytest.raises(ValueError, match="MG_MAX_LDS_DS"):
        jit.program_asm(prog, default_leafgen(prog), 16, ".Ljp0", 10)
    text = "\n".join(jit.program_asm(prog, default_leafgen(prog), 16, ".Ljp0", 8))
    offs = [int(m) for m in re.findall(r"\bds_\w+ .*offset:(\d+)", text)]
    assert offs and max(offs) <= 0xFFFF
    env = dict(os.environ, MYTHGPU_LDS_SLOTS="10")
    env.pop("MYTHGPU_NREG", None)
    r = subprocess.run([sys.executable, "-c", "from mythril_amd.engine import lds_slots_for; "
                        "lds_slots_for(16)"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "MG_MAX_LDS_DS" in r.stderr
