"""Build the oracle's C restatement (test infrastructure / CPU baseline):
oracle/lib/libevalref.so.  No -march=native: the .so travels to the GPU box."""

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "lib", "libevalref.so")


def build(force: bool = False) -> str:
    src = os.path.join(HERE, "evalref.c")
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= os.path.getmtime(src):
        return LIB
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.run(["gcc", "-O3", "-fopenmp", "-fPIC", "-shared", "-Wall", "-o", LIB + ".tmp", src],
                   check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force=True))
