"""Parity over the WHOLE bench configuration, not a sample.

``bench.py`` times ``mg_batch_eval_gen`` over every DAG of a workload (C2:
4096 corpus DAGs; C3 / C4: 256 distinct stand-in queries).  Here the same
entry point runs over every one of them at a 2^12-lane slice from a nonzero
first index, and every root bit and every per-DAG first satisfying index is
compared with ``oracle/evalref.c`` (``run_gen``: the same generator, the same
pools; pinned to ``oracle/smtlib_ref.py`` by tests/test_evalref.py).

The interpreter selects among up to 64 handler variants per opcode from
static properties, so the test also asserts that every
(family, variant) the bench configurations execute — reported by the
translator itself (``engine.handler_variants``) — belongs to a program this
test checked lane by lane.

The module runs on the register layout of its process (``MYTHGPU_NREG``):
the default 16 slots, and — from ``tests/test_gpu_layout.py``, in a fresh
process with ``MYTHGPU_NREG=11`` — the four-wave 11-slot layout that
``bench.py`` runs C2 on (the library's second interpreter, chosen by the
context: ``Engine(nreg=11)``).  Programs are compiled for the layout's slots
and translated for its LDS regions.
"""

import ctypes as C
import os

import numpy as np
import pytest

import bench
from mythril_amd import irdefs, shard
from mythril_amd.build import LAYOUT_LDS_SLOTS
from mythril_amd.engine import default_leafgen, handler_variants, unpack_bits

pytestmark = pytest.mark.gpu
THREADS = int(os.environ.get("OMP_NUM_THREADS", "0")) or 8
N_LANES, FIRST = 1 << 12, (3 << 20) + 192
SEED = bench.SEED
FULL = {w: bench.default_units(w) for w in ("c2", "c3", "c4", "c5")}
# (family, variant) handlers of the programs verified lane by lane below
CHECKED = set()
# the LDS spill regions of this process's layout (the context's)
LDS = int(os.environ.get("MYTHGPU_LDS_SLOTS", LAYOUT_LDS_SLOTS[irdefs.NREG]))


def test_layout_of_this_process(engine):
    """The context, the compiler and the translator agree on one layout."""
    from mythril_amd import asmgen
    assert engine.nreg == irdefs.NREG and engine.lds_slots == LDS == LAYOUT_LDS_SLOTS[irdefs.NREG]
    with asmgen.layout(irdefs.NREG):
        assert engine.lib.mg_asm_digest_layout(irdefs.NREG).decode() == asmgen.digest()
    _, p, _, _ = bench.compile_unit(("c2", 0))
    assert p.nreg == irdefs.NREG
    print("layout: %d slots, %d LDS regions, %s" % (irdefs.NREG, LDS,
                                                     os.path.basename(bench.engine_lib_path())))


def _oracle_unit(item):
    """Worker (spawned: no GPU state): compile one bench unit and evaluate it
    with the C oracle on the test's lane slice."""
    from oracle import evalref
    workload, d = item
    d, prog, _, _ = bench.compile_unit((workload, d))
    roots = bench.workload_roots(workload, d)
    want = evalref.run_gen(evalref.serialize(roots, prog), prog, SEED, d, FIRST, N_LANES, 1)
    return d, prog, np.packbits(want, bitorder="little")


@pytest.fixture(scope="module")
def units():
    """Every bench unit of C2, C3 and C4 with its oracle root bits (spawned
    workers: this process may already hold the GPU)."""
    from mythril_amd.procmap import process_map
    out = {}
    for w, n in FULL.items():
        # a worker that dies (an abort in the C oracle) raises
        # BrokenProcessPool at once instead of hanging the module (round 4)
        out[w] = sorted(process_map(_oracle_unit, [(w, d) for d in range(n)],
                                    min(16, os.cpu_count() or 1), "spawn", chunksize=8),
                        key=lambda t: t[0])
    return out


def _run_batch(engine, progs, image=None):
    hip = C.CDLL("libamdhip64.so.7")
    loaded = [engine.load(p, default_leafgen(p), prog_seed=d) for d, p in progs]
    jit_h = engine.jit_attach(loaded, image) if image is not None else None
    batch = engine.batch_create(loaded)
    bits = np.zeros((len(progs), N_LANES // 64), dtype=np.uint64)
    firsts = np.full(len(progs), shard.NONE, dtype=np.int64)
    d_bits, d_first = C.c_void_p(), C.c_void_p()
    assert hip.hipMalloc(C.byref(d_bits), C.c_size_t(bits.nbytes)) == 0
    assert hip.hipMalloc(C.byref(d_first), C.c_size_t(firsts.nbytes)) == 0
    try:
        assert hip.hipMemcpy(d_first, firsts.ctypes.data_as(C.c_void_p),
                             C.c_size_t(firsts.nbytes), 1) == 0
        engine.batch_eval_gen(batch, SEED, FIRST, N_LANES, d_bits.value, d_first.value)
        assert hip.hipDeviceSynchronize() == 0
        assert hip.hipMemcpy(bits.ctypes.data_as(C.c_void_p), d_bits,
                             C.c_size_t(bits.nbytes), 2) == 0
        assert hip.hipMemcpy(firsts.ctypes.data_as(C.c_void_p), d_first,
                             C.c_size_t(firsts.nbytes), 2) == 0
    finally:
        engine.batch_free(batch)
        if jit_h is not None:
            engine.jit_detach(jit_h)
        hip.hipFree(d_bits)
        hip.hipFree(d_first)
    return bits, firsts.tolist()


@pytest.fixture(scope="module")
def images(units):
    """Compiled-program code objects of every bench unit (bench.py --jit),
    built on spawned workers."""
    from mythril_amd import jit
    return {w: jit.compile_batch([(p, None, d) for d, p, _ in units[w]], workers=16,
                                 start="spawn", lds_slots=LDS) for w in FULL}


@pytest.mark.parametrize("path", ["interp", "jit"])
@pytest.mark.parametrize("workload", ["c2", "c3", "c4", "c5"])
def test_every_bench_unit_every_lane(engine, units, images, workload, path):
    us = units[workload]
    assert len(us) == FULL[workload]
    bits, firsts = _run_batch(engine, [(d, p) for d, p, _ in us],
                              images[workload] if path == "jit" else None)
    n_sat = n_hit = 0
    for k, (d, p, packed) in enumerate(us):
        want = np.unpackbits(packed, bitorder="little")[:N_LANES].astype(bool)
        got = unpack_bits(bits[k], N_LANES)
        assert np.array_equal(got, want), (workload, path, d, int(np.argmax(got != want)))
        hit = np.flatnonzero(want)
        assert firsts[k] == (FIRST + int(hit[0]) if hit.size else shard.NONE), (workload, d)
        n_sat += int(hit.size)
        n_hit += bool(hit.size)
    if path == "interp":
        for d, p, _ in us:
            CHECKED.update(handler_variants(p, LDS))
    print("%s %s: %d units, %d with satisfying lanes, %d satisfying lanes"
          % (workload, path, len(us), n_hit, n_sat))


def test_bench_handler_variants_all_checked(units):
    """Every (family, variant) executed by a bench configuration (what
    bench.py compiles for C2, C3, C4 and C5) belongs to a program the test above
    verified lane by lane; the count is reported so a new variant shows up
    in the log."""
    assert CHECKED, "run with test_every_bench_unit_every_lane (same module)"
    bench_set = set()
    for w in FULL:                      # the programs bench.compile_unit builds
        for d, p, _ in units[w]:
            bench_set |= handler_variants(p, LDS)
    missing = sorted(bench_set - CHECKED)
    assert not missing, missing
    fams = sorted({f for f, _ in bench_set})
    print("bench configurations execute %d (family, variant) handlers in %d families "
          "(%d-slot layout)" % (len(bench_set), len(fams), irdefs.NREG))


def test_jit_attach_refuses_code_compiled_for_other_records(engine):
    """mg_jit_attach compares each table row's record fingerprint with the
    loaded program's: an image compiled for another program (or another
    allocation of the same DAG) is refused, never entered."""
    from mythril_amd import jit
    from mythril_amd.engine import EngineError
    d1, p1, _, _ = bench.compile_unit(("c2", 1))
    d2, p2, _, _ = bench.compile_unit(("c2", 2))
    image = jit.compile_batch([(p1, None, d1)])
    lp2 = engine.load(p2, default_leafgen(p2), prog_seed=d2)
    with pytest.raises(EngineError, match="other records"):
        engine.jit_attach([lp2], image)
    lp1 = engine.load(p1, default_leafgen(p1), prog_seed=d1 + 1)     # another salt
    with pytest.raises(EngineError, match="other records"):
        engine.jit_attach([lp1], image)
    lp1 = engine.load(p1, default_leafgen(p1), prog_seed=d1)
    engine.jit_detach(engine.jit_attach([lp1], image))


def test_program_freed_while_attached_leaves_its_image(engine):
    """A program freed before its image is detached drops out of the image's
    list (mg_free_program), so the detach cannot write into the device block
    the next program reuses: that program keeps evaluating like the
    interpreter did before the detach."""
    from mythril_amd import jit
    d1, p1, _, _ = bench.compile_unit(("c2", 1))
    d2, p2, _, _ = bench.compile_unit(("c2", 2))
    image = jit.compile_batch([(p1, None, d1)])
    lp1 = engine.load(p1, default_leafgen(p1), prog_seed=d1)
    h = engine.jit_attach([lp1], image)
    del lp1                                       # freed while attached
    lp2 = engine.load(p2, default_leafgen(p2), prog_seed=d2)
    before = engine.eval_gen(lp2, bench.SEED, 5, 4096, want_probes=True)
    engine.jit_detach(h)
    after = engine.eval_gen(lp2, bench.SEED, 5, 4096, want_probes=True)
    assert np.array_equal(before[0], after[0])
    assert (before[1] is None and after[1] is None) or np.array_equal(before[1], after[1])


def test_jit_attach_refuses_an_opcode_twin(engine):
    """programs whose records differ only in an operation (ADD vs
    XOR, the handler id in word 0) must not share a fingerprint: the image of
    one is refused for the other, and accepted for itself."""
    from mythril_amd import jit
    from mythril_amd.engine import EngineError
    from test_jit import opcode_twins
    p_add, p_xor = opcode_twins()
    image = jit.compile_batch([(p_add, None, 1)])
    with pytest.raises(EngineError, match="other records"):
        engine.jit_attach([engine.load(p_xor, default_leafgen(p_xor), prog_seed=1)], image)
    lp = engine.load(p_add, default_leafgen(p_add), prog_seed=1)
    engine.jit_detach(engine.jit_attach([lp], image))


def test_jit_attach_refuses_another_interpreter_and_stray_entries(engine, monkeypatch):
    """The table header carries the asm digest of the interpreter the code
    was generated for (pinned registers, descriptor layout): an image made
    for another one is refused.  An entry pointing outside the image's
    executable sections (here: into the table itself) is refused too."""
    from mythril_amd import jit
    from mythril_amd.engine import EngineError
    d1, p1, _, _ = bench.compile_unit(("c2", 1))
    lp = engine.load(p1, default_leafgen(p1), prog_seed=d1)
    real = jit.table_asm
    monkeypatch.setattr(jit.G, "digest", lambda *a: "0123456789abcdef")
    stale = jit.compile_batch([(p1, None, d1)])
    monkeypatch.undo()
    with pytest.raises(EngineError, match="another interpreter"):
        engine.jit_attach([lp], stale)

    def stray(fps, nreg=None):
        return real(fps, nreg).replace("\t.quad mg_jp0 - . + 16\n", "\t.quad 16\n")
    monkeypatch.setattr(jit, "table_asm", stray)
    bad = jit.compile_batch([(p1, None, d1)])
    monkeypatch.undo()
    with pytest.raises(EngineError, match="outside the code"):
        engine.jit_attach([lp], bad)
    engine.jit_detach(engine.jit_attach([lp], jit.compile_batch([(p1, None, d1)])))


def test_free_waits_for_launches_on_every_caller_stream(engine):
    """a long batch queued on caller stream A, then a short one on
    stream B; the first batch and its programs are freed at once and new
    programs are loaded into the recycled device blocks.  The free must wait
    for A too (not only the last stream), so A's results equal a clean run."""
    hip = C.CDLL("libamdhip64.so.7")
    ids_a, ids_b, ids_c = range(0, 48), range(48, 50), range(100, 148)
    progs = {d: bench.compile_unit(("c2", d))[1] for d in list(ids_a) + list(ids_b) + list(ids_c)}
    n = 1 << 17
    words = n // 64

    def run_on(stream, ids, d_bits, d_first, free_after=False):
        loaded = [engine.load(progs[d], default_leafgen(progs[d]), prog_seed=d) for d in ids]
        batch = engine.batch_create(loaded)
        engine.batch_eval_gen(batch, SEED, 7, n, d_bits, d_first, stream)
        return loaded, batch

    def dev(nbytes):
        p = C.c_void_p()
        assert hip.hipMalloc(C.byref(p), C.c_size_t(nbytes)) == 0
        return p

    bits_a, first_a = dev(len(ids_a) * words * 8), dev(len(ids_a) * 8)
    bits_b, first_b = dev(len(ids_b) * words * 8), dev(len(ids_b) * 8)
    sa, sb = C.c_void_p(), C.c_void_p()
    assert hip.hipStreamCreate(C.byref(sa)) == 0 and hip.hipStreamCreate(C.byref(sb)) == 0
    try:
        ones = np.full(len(ids_a), shard.NONE, dtype=np.int64)
        # reference: the same batch alone, completed
        assert hip.hipMemcpy(first_a, ones.ctypes.data_as(C.c_void_p), C.c_size_t(ones.nbytes), 1) == 0
        la, ba = run_on(sa.value, ids_a, bits_a.value, first_a.value)
        assert hip.hipStreamSynchronize(sa) == 0
        want = np.zeros((len(ids_a), words), dtype=np.uint64)
        assert hip.hipMemcpy(want.ctypes.data_as(C.c_void_p), bits_a, C.c_size_t(want.nbytes), 2) == 0
        engine.batch_free(ba)
        del la
        # the race: A long, B short, free A's blocks, reuse them at once
        assert hip.hipMemsetAsync(bits_a, 0, C.c_size_t(want.nbytes), sa) == 0
        la, ba = run_on(sa.value, ids_a, bits_a.value, first_a.value)
        lb, bb = run_on(sb.value, ids_b, bits_b.value, first_b.value)
        engine.batch_free(ba)
        del la
        lc = [engine.load(progs[d], default_leafgen(progs[d]), prog_seed=d) for d in ids_c]
        assert hip.hipDeviceSynchronize() == 0
        got = np.zeros_like(want)
        assert hip.hipMemcpy(got.ctypes.data_as(C.c_void_p), bits_a, C.c_size_t(got.nbytes), 2) == 0
        assert np.array_equal(got, want)
        engine.batch_free(bb)
        del lb, lc
    finally:
        for p in (bits_a, first_a, bits_b, first_b):
            hip.hipFree(p)
        hip.hipStreamDestroy(sa)
        hip.hipStreamDestroy(sb)
