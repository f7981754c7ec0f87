"""Build the oracle's C restatement (test infrastructure / CPU baseline):
oracle/lib/libevalref.so.  No -march=native: the .so travels to the GPU box."""

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "lib", "libevalref.so")
LIB_WIDE = os.path.join(HERE, "lib", "libevalref_wide.so")    # 1024-bit values (-DL=16)


def build(force: bool = False) -> str:
    src = os.path.join(HERE, "evalref.c")
    for lib, defs in ((LIB, []), (LIB_WIDE, ["-DL=16"])):
        if not force and os.path.exists(lib) and os.path.getmtime(lib) >= os.path.getmtime(src):
            continue
        os.makedirs(os.path.dirname(lib), exist_ok=True)
        subprocess.run(["gcc", "-O3", "-fopenmp", "-fPIC", "-shared", "-Wall"] + defs +
                       ["-o", lib + ".tmp", src], check=True)
        os.replace(lib + ".tmp", lib)
    return LIB


if __name__ == "__main__":
    print(build(force=True))
