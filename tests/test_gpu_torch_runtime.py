"""The configuration bench.py times: PyTorch imported FIRST, so the library's
``NEEDED libamdhip64.so.7`` binds to the HIP runtime torch bundles (not
/opt/rocm's, which every other GPU test runs on), device buffers are torch
tensors and the launches go to a torch stream.  A child process (fresh, so
torch really is first) runs ``mg_batch_eval_gen`` exactly as bench.py's step
does — compiled programs and the interpreter — and every root bit and
per-DAG first satisfying index is compared with ``oracle/evalref.c``."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, sys
import numpy as np
import torch                                   # first: its libamdhip64 wins
torch.cuda.set_device(0)
sys.path.insert(0, %(root)r)
import bench
from mythril_amd import jit, shard
from mythril_amd.engine import Engine, default_leafgen, unpack_bits
from oracle import evalref
ids = list(range(0, 4096, 128))
corpus = [bench.compile_unit(("c2", d)) for d in ids]
eng = Engine(0)
n, first = 1 << 14, (5 << 20) + 64
out = {"runtime": eng.runtime_info(), "torch_hip": torch.version.hip, "paths": {}}
for path in ("jit", "interp"):
    loaded = [eng.load(p, default_leafgen(p), prog_seed=d) for d, p, _, _ in corpus]
    h = eng.jit_attach(loaded, jit.compile_batch([(p, None, d) for d, p, _, _ in corpus])) \
        if path == "jit" else None
    batch = eng.batch_create(loaded)
    bits = torch.zeros((len(ids), n // 64), dtype=torch.int64, device="cuda")
    firsts = torch.full((len(ids),), shard.NONE, dtype=torch.int64, device="cuda")
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    eng.batch_eval_gen(batch, bench.SEED, first, n, bits.data_ptr(), firsts.data_ptr(),
                       stream.cuda_stream)
    torch.cuda.synchronize()
    rows, fs = bits.cpu().numpy().view(np.uint64), firsts.cpu().tolist()
    bad = badf = 0
    for k, (d, p, _, _) in enumerate(corpus):
        want = evalref.run_gen(evalref.serialize(bench.workload_roots("c2", d), p), p,
                               bench.SEED, d, first, n, 8)
        bad += int(np.count_nonzero(unpack_bits(rows[k], n) != want))
        hit = np.flatnonzero(want)
        badf += fs[k] != (first + int(hit[0]) if hit.size else shard.NONE)
    out["paths"][path] = {"mismatches": bad, "first_mismatches": badf}
    eng.batch_free(batch)
    if h is not None:
        eng.jit_detach(h)
print("RESULT " + json.dumps(out))
'''


def test_parity_on_torchs_runtime_with_torch_buffers_and_stream():
    env = dict(os.environ)
    r = subprocess.run([sys.executable, "-c", CHILD % {"root": ROOT}], capture_output=True,
                       text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = next(l for l in r.stdout.splitlines() if l.startswith("RESULT "))
    res = json.loads(line[len("RESULT "):])
    print(res)
    for path, got in res["paths"].items():
        assert got == {"mismatches": 0, "first_mismatches": 0}, (path, got)
    assert res["runtime"]["hip_runtime_version"] > 0
    # the runtime really is torch's bundled one in this configuration
    assert "torch" in res["runtime"]["libamdhip64"], res["runtime"]
