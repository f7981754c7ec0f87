"""Build libmythgpu.so in-tree (hipcc, gfx950): the interpreter of every
register layout, the Keccak kernel and the host code in one library.  The
.so travels to the GPU box with the repo snapshot; nothing is JIT-compiled at
run time."""

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

# Register layouts (mg_layouts in mg_host.cpp): slots ->
# (waves per SIMD, default LDS spill regions).  ONE library holds the
# interpreter of each: mg_interp_asm.hip is compiled once per layout, the
# 16-slot body from the tracked generated sources, the others from a private
# copy of csrc/ that asmgen fills for their slot count; a context runs one
# layout (mg_init_layout), chosen per batch (mythril_amd/layout.py).
LAYOUTS = {16: (3, 6), 11: (4, 5)}
LAYOUT_LDS_SLOTS = {n: lds for n, (_, lds) in LAYOUTS.items()}


def _hipcc(csrc: str, src: str, obj: str, defines=(), flags=None, verbose: bool = False):
    cmd = [HIPCC, "--offload-arch=" + ARCH] + (HIP_FLAGS if flags is None else flags) + \
          ["-D" + d for d in defines] + [
           "-I" + csrc, "-I" + os.path.join(ROOT, "include"), "-c", os.path.join(csrc, src),
           "-o", obj]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return obj


def _generate(nreg: int, dst: str) -> None:
    """asmgen's outputs for a ``nreg``-slot layout into ``dst``."""
    from mythril_amd import asmgen
    with asmgen.layout(nreg):
        asmgen.write_outputs(dst)


def build(force: bool = False, verbose: bool = False, out: str = LIB, defines=(),
          flags=None) -> str:
    if not force and out == LIB and up_to_date():
        return LIB
    os.makedirs(os.path.dirname(out), exist_ok=True)
    import shutil
    import tempfile
    # the 16-slot interpreter's body and handler numbering are generated into
    # the tracked sources (whatever this process's MYTHGPU_NREG)
    _generate(16, CSRC)
    objs = []
    with tempfile.TemporaryDirectory() as td:
        for src in SOURCES:
            objs.append(_hipcc(CSRC, src, os.path.join(td, src + ".o"), defines, flags, verbose))
        for nreg, (waves, _) in sorted(LAYOUTS.items()):
            if nreg == 16:
                continue
            lay = os.path.join(td, "csrc_r%d" % nreg)
            shutil.copytree(CSRC, lay)
            _generate(nreg, lay)
            objs.append(_hipcc(lay, "mg_interp_asm.hip", os.path.join(td, "interp_r%d.o" % nreg),
                               list(defines) + ["MG_LAYOUT_NREG=%d" % nreg,
                                                "MG_ASM_WAVES_PER_SIMD=%d" % waves],
                               flags, verbose))
        tmp = out + ".tmp"
        subprocess.run([HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", tmp] + objs,
                       check=True)
        os.replace(tmp, out)
    if out == LIB:
        build_jit_stub()
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
    print(build_compiler(force="--force" in sys.argv))
