"""The four-wave register layout (11 slots: the library's second
interpreter) that bench.py runs the C2 corpus on (chosen per batch by
mythril_amd/layout.py): a small default-shaped C2 bench whose
self-check compares the root bits and first satisfying indices of its own
launch with oracle/evalref.c; the whole bench configuration on that layout;
and both layouts launched from one process."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_c2_four_wave_layout_self_check():
    env = dict(os.environ)
    for k in ("MYTHGPU_NREG", "MYTHGPU_LDS_SLOTS", "MYTHGPU_LIB", "MYTHGPU_JIT_CACHE"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-u", "bench.py", "--workload", "c2", "--dags", "256",
                        "--steps", "1", "--warmup", "0", "--assign-log2", "16"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    d = json.loads(r.stdout[r.stdout.rindex('{"metric"'):])
    assert d["config"]["register_layout"] == "11 slots, 4 waves/SIMD, 5 LDS regions"
    assert d["config"]["layout_rule"]["nreg"] == 11 and not d["config"]["layout_rule"]["explicit"]
    assert d["runtime"]["library"] == "libmythgpu.so"
    sc = d["selfcheck"]
    assert sc["dags"] > 0 and sc["lanes"] > 0
    assert sc["mismatches"] == 0 and sc["first_sat_mismatches"] == 0


@pytest.mark.gpu
def test_four_wave_layout_whole_bench_configuration():
    """the whole-configuration parity of
    test_gpu_bench_parity.py — every bench unit of C2 (4096 DAGs), C3, C4
    and C5, 2^12 lanes each, interpreter and compiled programs, root bits and
    first satisfying indices against oracle/evalref.c, plus the handler-variant
    coverage — on the four-wave layout, in a fresh process whose compiler,
    translator and library are the 11-slot ones (the layout is chosen before
    anything imports the compiler).  The module itself asserts that the
    context runs 11 slots and 5 LDS regions."""
    env = dict(os.environ, MYTHGPU_NREG="11")
    for k in ("MYTHGPU_LIB", "MYTHGPU_JIT_CACHE", "PYTEST_ADDOPTS", "MYTHGPU_LDS_SLOTS"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-u", "-m", "pytest", "tests/test_gpu_bench_parity.py",
                        "-m", "gpu", "-q", "-s", "-p", "no:cacheprovider",
                        "-k", "layout_of_this_process or every_bench_unit or handler_variants"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    out = r.stdout
    print(out[-3000:])
    assert r.returncode == 0, (out[-3000:], r.stderr[-3000:])
    assert "layout: 11 slots, 5 LDS regions, libmythgpu.so" in out
    assert "10 passed" in out
    assert "(11-slot layout)" in out
    for w in ("c2", "c3", "c4", "c5"):
        for path in ("interp", "jit"):
            assert "%s %s: " % (w, path) in out, (w, path)


@pytest.mark.gpu
def test_both_layouts_in_one_process():
    """one process, one library, two contexts — the
    16-slot and the 11-slot interpreter — each launched on a batch compiled
    for it (interpreted and compiled code); both give the oracle's root bits
    and first satisfying indices, a program of one layout is refused by the
    other's context, and the layout rule picks 11 for the C2 batch and 16 for
    the C3 batch."""
    import numpy as np
    import bench
    from mythril_amd import jit, layout, shard
    from mythril_amd.engine import EngineError, get_engine
    from mythril_amd.procmap import process_map
    from test_gpu_bench_parity import FIRST, N_LANES, SEED, _run_batch

    units = [("c2", d) for d in range(0, 4096, 256)] + [("c3", d) for d in range(0, 256, 32)]
    want = dict(process_map(_oracle_ref, units, 8, "spawn"))
    e16, e11 = get_engine(0, nreg=16), get_engine(0, nreg=11)
    assert (e16.nreg, e11.nreg, e16.lds_slots, e11.lds_slots) == (16, 11, 6, 5)
    for w in ("c2", "c3"):
        ids = [d for ww, d in units if ww == w]
        p16 = [bench.compile_unit((w, d, 16))[1] for d in ids]
        assert layout.choose(p16) == (11 if w == "c2" else 16)
        for nreg, eng in ((16, e16), (11, e11)):
            progs = [(d, bench.compile_unit((w, d, nreg))[1]) for d in ids]
            images = [None, jit.compile_batch([(p, None, d) for d, p in progs])]
            for image in images:
                bits, firsts = _run_batch(eng, progs, image)
                for k, d in enumerate(ids):
                    wb = want[(w, d)]
                    got = np.unpackbits(bits[k].view(np.uint8), bitorder="little")[:N_LANES]
                    assert np.array_equal(got.astype(bool), wb), (w, d, nreg, image is not None)
                    hit = np.flatnonzero(wb)
                    assert firsts[k] == (FIRST + int(hit[0]) if hit.size else shard.NONE)
    p16 = bench.compile_unit(("c2", 0, 16))[1]
    with pytest.raises(EngineError, match="register slots"):
        e11.load(p16)


def _oracle_ref(item):
    """(workload, unit) -> its oracle root bits on test_gpu_bench_parity's
    lane slice (a spawned worker: no GPU state)."""
    import numpy as np
    import bench
    from oracle import evalref
    from test_gpu_bench_parity import FIRST, N_LANES, SEED
    w, d = item
    _, prog, _, _ = bench.compile_unit((w, d, 16))
    roots = bench.workload_roots(w, d)
    bits = evalref.run_gen(evalref.serialize(roots, prog), prog, SEED, d, FIRST, N_LANES, 1)
    return item, np.asarray(bits, dtype=bool)[:N_LANES]
