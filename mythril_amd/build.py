"""Build libmythgpu.so in-tree (hipcc, gfx950).  The .so travels to the GPU
box with the repo snapshot; nothing is JIT-compiled at run time."""

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mythril_amd", "csrc")
LIBDIR = os.path.join(ROOT, "mythril_amd", "lib")
LIB = os.path.join(LIBDIR, "libmythgpu.so")
JIT_STUB = os.path.join(LIBDIR, "mg_jit_stub.s")
SOURCES = ["mg_interp_asm.hip", "mg_keccak.hip", "mg_host.cpp", "mg_api.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("MYTHGPU_ARCH", "gfx950")


def _deps():
    files = [os.path.join(CSRC, s) for s in SOURCES]
    files += [os.path.join(CSRC, "mg_device.h"), os.path.join(CSRC, "mg_host.h"),
              os.path.join(CSRC, "mg_jit_stub.hip"),
              os.path.join(ROOT, "include", "mythgpu.h"),
              os.path.join(ROOT, "include", "mythgpu_ir.h"),
              os.path.join(ROOT, "mythril_amd", "asmgen.py")]
    return files


def up_to_date() -> bool:
    if not os.path.exists(LIB) or not os.path.exists(JIT_STUB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(f) <= t for f in _deps())


# Keep uniform (wave-uniform) control flow unstructured: the opcode switch
# then lowers to a plain scalar binary search with direct branches instead
# of structurizer "Flow" blocks on every join (fewer SALU per instruction).
HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-mllvm", "-structurizecfg-skip-uniform-regions=true"]


def _compile(csrc: str, out: str, defines=(), flags=None, verbose: bool = False) -> str:
    objs = []
    for src in SOURCES:
        obj = out + "." + src + ".o"
        cmd = [HIPCC, "--offload-arch=" + ARCH] + (HIP_FLAGS if flags is None else flags) + \
              ["-D" + d for d in defines] + [
               "-I" + os.path.join(ROOT, "include"), "-I" + csrc, "-c",
               os.path.join(csrc, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        objs.append(obj)
    tmp = out + ".tmp"
    subprocess.run([HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", tmp] + objs,
                   check=True)
    os.replace(tmp, out)
    for o in objs:
        os.remove(o)
    return out


def build(force: bool = False, verbose: bool = False, out: str = LIB, defines=(),
          flags=None) -> str:
    if not force and out == LIB and up_to_date():
        return LIB
    os.makedirs(os.path.dirname(out), exist_ok=True)
    # the assembly interpreter's body and handler numbering are generated —
    # for the default 16-slot layout whatever this process's MYTHGPU_NREG
    # (an 11-slot generator would overwrite the tracked sources
    # and pair 11-slot handlers with the C code's 16 slots)
    _generate(16, CSRC)
    _compile(CSRC, out, defines, flags, verbose)
    if out == LIB:
        build_jit_stub()
    return out


# Register layouts: 16 slots at three waves per SIMD (the
# default library) and 11 slots at four (128 VGPRs, five LDS regions of
# 40 KiB per block).  A layout other than 16 is generated under
# MYTHGPU_NREG into a private copy of csrc/, so the tracked generated files
# stay the default's.
LIB_W4 = os.path.join(LIBDIR, "libmythgpu_w4.so")
LAYOUTS = {16: (LIB, ()),
           11: (LIB_W4, ("MG_NREG_OVERRIDE=11", "MG_ASM_WAVES_PER_SIMD=4",
                         "MG_LDS_SLOTS_DEFAULT=5"))}
LAYOUT_LDS_SLOTS = {16: 6, 11: 5}


def lib_for_layout(nreg: int) -> str:
    if nreg not in LAYOUTS:
        raise ValueError("no library for a %d-slot register layout (have %s)"
                         % (nreg, sorted(LAYOUTS)))
    return LAYOUTS[nreg][0]


def _generate(nreg: int, dst: str) -> None:
    """asmgen's outputs for a ``nreg``-slot layout into ``dst`` (in this
    process when its generator already has that layout, else in a child
    with MYTHGPU_NREG set to it)."""
    from mythril_amd import asmgen
    if asmgen.NREG == nreg:
        asmgen.write_outputs(dst)
        return
    code = ("import sys; sys.path.insert(0, %r); from mythril_amd import asmgen; "
            "assert asmgen.NREG == %d; asmgen.write_outputs(%r)" % (ROOT, nreg, dst))
    subprocess.run([sys.executable, "-c", code], check=True,
                   env=dict(os.environ, MYTHGPU_NREG=str(nreg)))


def build_layout(nreg: int, force: bool = False, verbose: bool = False) -> str:
    out, defines = LAYOUTS[nreg]
    if nreg == 16:
        return build(force, verbose)
    if not force and _fresh(out, _deps()):
        return out
    import shutil
    import tempfile
    os.makedirs(LIBDIR, exist_ok=True)
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "csrc")
        shutil.copytree(CSRC, src)
        _generate(nreg, src)
        _compile(src, out, defines, None, verbose)
    return out


def build_jit_stub() -> str:
    """Device assembly of the stub kernel every compiled-program code object
    (mythril_amd/jit.py) is built around."""
    tmp = JIT_STUB + ".tmp"
    subprocess.run([HIPCC, "--offload-arch=" + ARCH, "-O3", "--cuda-device-only", "-S",
                    os.path.join(CSRC, "mg_jit_stub.hip"), "-o", tmp], check=True,
                   stderr=subprocess.DEVNULL)
    os.replace(tmp, JIT_STUB)
    return JIT_STUB


CC_LIB = os.path.join(LIBDIR, "libmythcc.so")
CC_SOURCES = [os.path.join(CSRC, "mg_compile.cpp"), os.path.join(ROOT, "include", "mythcc.h"),
              os.path.join(ROOT, "include", "mythgpu_ir.h")]
CC_PY_SOURCE = os.path.join(CSRC, "mg_compile_py.cpp")


def cc_ext_path() -> str:
    import sysconfig
    return os.path.join(LIBDIR, "_mythcc" + sysconfig.get_config_var("EXT_SUFFIX"))


def _fresh(out, deps) -> bool:
    return os.path.exists(out) and all(os.path.getmtime(f) <= os.path.getmtime(out) for f in deps)


def build_compiler(force: bool = False) -> str:
    """The native host compiler (include/mythcc.h, plain host C++, g++): the
    C-ABI library libmythcc.so and the CPython front-end _mythcc (the same
    compiler plus a DAG walk over the Python objects)."""
    import sysconfig
    os.makedirs(LIBDIR, exist_ok=True)
    flags = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-I" + os.path.join(ROOT, "include")]
    if force or not _fresh(CC_LIB, CC_SOURCES):
        tmp = "%s.%d.tmp" % (CC_LIB, os.getpid())
        subprocess.run(flags + [CC_SOURCES[0], "-o", tmp], check=True)
        os.replace(tmp, CC_LIB)
    ext = cc_ext_path()
    if force or not _fresh(ext, CC_SOURCES + [CC_PY_SOURCE]):
        tmp = "%s.%d.tmp" % (ext, os.getpid())
        subprocess.run(flags + ["-I" + sysconfig.get_paths()["include"], CC_PY_SOURCE, CC_SOURCES[0],
                                "-o", tmp], check=True)
        os.replace(tmp, ext)
    return CC_LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    print(build_layout(11, force="--force" in sys.argv))
    print(build_compiler(force="--force" in sys.argv))
