#!/usr/bin/env python3
"""First GPU contact of a compiled-program build: a few corpus DAGs through
mg_batch_eval_gen on the interpreter and on their compiled code; root bits
and first indices must be identical.  Exits non-zero on any difference."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from mythril_amd import jit, shard  # noqa: E402

n_dags = int(sys.argv[1]) if len(sys.argv) > 1 else 16
corpus = bench.build_corpus(n_dags, 8)
image = jit.compile_batch([(p, None, d) for d, p, _, _ in corpus], workers=8)
print("image %.1f MB" % (len(image) / 1e6), flush=True)

from mythril_amd.engine import Engine, default_leafgen  # noqa: E402
eng = Engine(0)
hip = C.CDLL("libamdhip64.so.7")
N, FIRST = 1 << 12, (3 << 20) + 192


def run(use_jit):
    loaded = [eng.load(p, default_leafgen(p), prog_seed=d) for d, p, _, _ in corpus]
    jh = eng.jit_attach(loaded, image) if use_jit else None
    b = eng.batch_create(loaded)
    bits = np.zeros((len(loaded), N // 64), dtype=np.uint64)
    first = np.full(len(loaded), shard.NONE, dtype=np.int64)
    db, df = C.c_void_p(), C.c_void_p()
    assert hip.hipMalloc(C.byref(db), C.c_size_t(bits.nbytes)) == 0
    assert hip.hipMalloc(C.byref(df), C.c_size_t(first.nbytes)) == 0
    assert hip.hipMemcpy(df, first.ctypes.data_as(C.c_void_p), C.c_size_t(first.nbytes), 1) == 0
    eng.batch_eval_gen(b, bench.SEED, FIRST, N, db.value, df.value)
    assert hip.hipDeviceSynchronize() == 0
    assert hip.hipMemcpy(bits.ctypes.data_as(C.c_void_p), db, C.c_size_t(bits.nbytes), 2) == 0
    assert hip.hipMemcpy(first.ctypes.data_as(C.c_void_p), df, C.c_size_t(first.nbytes), 2) == 0
    eng.batch_free(b)
    if jh is not None:
        eng.jit_detach(jh)
    hip.hipFree(db)
    hip.hipFree(df)
    return bits, first


bi, fi = run(False)
print("interpreter done", flush=True)
bj, fj = run(True)
print("jit done", flush=True)
same = np.array_equal(bi, bj) and np.array_equal(fi, fj)
print("identical:", same, "sat lanes", int(sum(bin(int(x)).count("1") for x in bi.reshape(-1))))
for k in range(len(corpus)):
    if not np.array_equal(bi[k], bj[k]):
        diff = np.flatnonzero(np.unpackbits((bi[k] ^ bj[k]).view(np.uint8), bitorder="little"))
        print("  dag", corpus[k][0], "lanes", diff[:10].tolist(), "interp bits",
              [int(bi[k][l // 64] >> (l % 64)) & 1 for l in diff[:10]])
sys.exit(0 if same else 1)
