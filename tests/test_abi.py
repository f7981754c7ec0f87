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


def test_four_wave_build_exports_the_same_abi():
    """libmythgpu_w4.so (bench's C2 layout) exports every declared symbol,
    reports 11 register slots, and was generated from the current generator
    under that layout (its digest, computed in a fresh process)."""
    import json
    import subprocess
    import sys
    lib = ctypes.CDLL(build.LIB_W4)
    for n in declared():
        assert hasattr(lib, n), n
    lib.mg_config.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32]
    cfg = (ctypes.c_uint32 * 4)()
    assert lib.mg_config(cfg, 4) == 0 and cfg[1] == 11
    lib.mg_asm_digest.restype = ctypes.c_char_p
    env = dict(os.environ, MYTHGPU_NREG="11")
    out = subprocess.run([sys.executable, "-c", "import json; from mythril_amd import asmgen; "
                          "print(json.dumps([asmgen.digest(), asmgen.NVGPR_KERNEL]))"],
                         cwd=build.ROOT, env=env, check=True, capture_output=True, text=True).stdout
    digest, nvgpr = json.loads(out.strip().splitlines()[-1])
    assert lib.mg_asm_digest().decode() == digest
    assert nvgpr == 128          # 512 / 128 = four waves per SIMD


def test_version_without_gpu():
    assert load_library().mg_version() == 3


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
                 "mg_last_kernel_ms", "mg_runtime_info", "mg_init"}
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
    # mg_init selects the device it is given
    assert "hipSetDevice(device)" in bodies["mg_init"]


def test_lds_regions_beyond_ds_offsets_are_refused_when_configured():
    """MYTHGPU_LDS_SLOTS=10 used to yield compiled code the
    assembler rejected (LDS halves past a DS instruction's 16-bit offset).
    Such a region count is refused where it is configured — the compiled-
    program renderer, bench.apply_layout and (header) mg_init — and the
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
    r = subprocess.run([sys.executable, "-c", "import bench; bench.apply_layout('c3')"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "MG_MAX_LDS_DS" in r.stderr
