"""The four-wave register layout (11 slots, libmythgpu_w4.so) that
bench.py runs the C2 corpus on (bench.WORKLOAD_NREG): a small
default-shaped C2 bench in a fresh process (the layout is chosen before the
compiler is imported) whose self-check compares the root bits and first
satisfying indices of its own launch with oracle/evalref.c.  The 16-slot
layout's parity is test_gpu_bench_parity.py's."""
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
    assert d["runtime"]["library"] == "libmythgpu_w4.so"
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
    library is libmythgpu_w4.so with 11 slots and 5 LDS regions."""
    env = dict(os.environ, MYTHGPU_NREG="11", MYTHGPU_LDS_SLOTS="5")
    for k in ("MYTHGPU_LIB", "MYTHGPU_JIT_CACHE", "PYTEST_ADDOPTS"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-u", "-m", "pytest", "tests/test_gpu_bench_parity.py",
                        "-m", "gpu", "-q", "-s", "-p", "no:cacheprovider",
                        "-k", "layout_of_this_process or every_bench_unit or handler_variants"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    out = r.stdout
    print(out[-3000:])
    assert r.returncode == 0, (out[-3000:], r.stderr[-3000:])
    assert "layout: 11 slots, 5 LDS regions, libmythgpu_w4.so" in out
    assert "10 passed" in out
    assert "(11-slot layout)" in out
    for w in ("c2", "c3", "c4", "c5"):
        for path in ("interp", "jit"):
            assert "%s %s: " % (w, path) in out, (w, path)
