"""Compiled programs (mythril_amd/jit.py) on the CPU: the straight-line code
generated for a program, run through the instruction-level simulator
(tests/asm_sim.py) exactly as the GPU enters it (the interpreter kernel's
body, the descriptor's jit_entry, s_swappc, shared division bodies), gives
the interpreter's results bit for bit and the oracle's values on every lane;
the code object assembles and its entry table points at each program."""

import random
import re
import subprocess

import numpy as np
import pytest

import asm_sim
import dag_cases
from mythril_amd import jit
from mythril_amd.assign import Assignment as PA, pack, unpack
from mythril_amd.corpus import make_dag
from mythril_amd.engine import default_leafgen, limbs_to_int
from mythril_amd.ir import compile_constraints
from oracle import smtlib_ref as R
from test_gpu_parity import flat_expected

CASES = dag_cases.named_cases()
SEED = 0x6D797468


@pytest.mark.parametrize("name", sorted(CASES))
def test_jit_case_equals_interpreter_and_oracle(name):
    constraints, probes, gen, tables = CASES[name]
    prog = compile_constraints(constraints, probes, table_sizes=tables)
    rng = random.Random(3000 + len(name))
    asgs = [gen(rng) for _ in range(64)]
    soa = pack(prog, [PA(a.vars, a.arrays, a.funcs) for a in asgs])
    r_i, pr_i, _, _ = asm_sim.simulate(prog, soa)
    r_j, pr_j, _, _ = asm_sim.simulate(prog, soa, jit=True)
    assert np.array_equal(pr_i, pr_j) and np.array_equal(r_i, r_j)
    for a, asg in enumerate(asgs):
        want = flat_expected(probes, R.evaluate(list(probes), asg))
        got = [limbs_to_int(pr_j[k, :, a]) for k in range(prog.n_probes)]
        assert got == want, a
        assert bool(r_j[a]) == bool(R.eval_constraints(constraints, asg)), a


@pytest.mark.parametrize("dag_id,n_lds", [(0, 6), (5, 6), (571, 6), (7, 2), (33, 0)])
def test_jit_corpus_dag_generator_mode(dag_id, n_lds):
    """Corpus DAGs with every constraint probed, device-generated leaves,
    spills split between LDS and scratch: interpreter == compiled, and the
    oracle agrees on every lane."""
    roots, _ = make_dag(dag_id, SEED)
    prog = compile_constraints([], roots)
    lg = default_leafgen(prog)
    first = 4096 + 77 * dag_id
    r_i, pr_i, lo_i, _ = asm_sim.simulate(prog, gen=(SEED, dag_id, first, lg), n_lds=n_lds,
                                          want_leaves=True)
    r_j, pr_j, lo_j, _ = asm_sim.simulate(prog, gen=(SEED, dag_id, first, lg), n_lds=n_lds,
                                          want_leaves=True, jit=True)
    assert np.array_equal(lo_i, lo_j) and np.array_equal(pr_i, pr_j) and np.array_equal(r_i, r_j)
    # no leaf store: compiled leaves take their one-flag common path
    # (asmgen.h_leafd, S_FAST); same roots and probes
    r_f, pr_f, _, _ = asm_sim.simulate(prog, gen=(SEED, dag_id, first, lg), n_lds=n_lds, jit=True)
    assert np.array_equal(pr_f, pr_j) and np.array_equal(r_f, r_j)
    for lane in range(0, 64, 7):
        asg = unpack(prog, lo_j[:, :, lane])
        want = R.evaluate(list(roots), R.Assignment(asg.vars, asg.arrays, asg.funcs))
        assert [int(pr_j[k, 0, lane]) for k in range(len(roots))] == [int(w) for w in want]


def test_jit_text_has_no_scalar_stores_and_fits_the_register_budget():
    roots, _ = make_dag(9, SEED)
    prog = compile_constraints(roots)
    text = jit.program_asm(prog, default_leafgen(prog), 9, ".Ljp0") + jit.bodies()
    for bad in ("s_store", "s_buffer_store", "s_scratch_store", "s_dcache", "s_atomic"):
        assert not any(bad in l for l in text)
    for l in text:
        for m in re.finditer(r"v\[?(\d+)", l):
            assert int(m.group(1)) < 168, l
    assert not any("s_set_gpr_idx" in l for l in jit.program_asm(prog, default_leafgen(prog), 9,
                                                                  ".Ljp1"))


def test_records_fingerprint_matches_the_c_definition():
    """records_fingerprint (numpy, wrapping uint64) against a plain restatement
    of mg_api.cpp's rec_fingerprint loop: every word, word 0 (the handler id)
    included."""
    rng = np.random.default_rng(5)
    rec = rng.integers(0, 1 << 32, size=8 * 37, dtype=np.uint64)
    h, p = 0, 1
    for r in range(0, len(rec), 8):
        for k in range(8):
            p = p * 0x100000001B3 % (1 << 64)
            h = (h + int(rec[r + k]) * p) % (1 << 64)
    assert jit.records_fingerprint(rec) == (h + 37) % (1 << 64)
    rec2 = rec.copy()
    rec2[8 * 5 + 3] ^= 1
    assert jit.records_fingerprint(rec2) != jit.records_fingerprint(rec)
    rec2 = rec.copy()
    rec2[8 * 5] ^= 1                          # word 0 (the handler id) is hashed
    assert jit.records_fingerprint(rec2) != jit.records_fingerprint(rec)


def opcode_twins():
    """Two programs whose records differ ONLY in one handler id (ADD vs XOR:
    same operands, same variant rules, no constants)."""
    from mythril_amd import smt
    x, y, z = (smt.symbol_factory.BitVecSym(n, 256) for n in "xyz")
    p_add = compile_constraints([((x + y) == z).raw])
    p_xor = compile_constraints([((x ^ y) == z).raw])
    return p_add, p_xor


def test_fingerprint_tells_opcode_twins_apart():
    """the fingerprint skipped word 0, so programs differing only
    in an opcode shared it and an image for one was accepted for the other."""
    from mythril_amd.engine import translate_records
    p_add, p_xor = opcode_twins()
    ra, _ = translate_records(p_add)
    rx, _ = translate_records(p_xor)
    ra, rx = ra.reshape(-1, 8), rx.reshape(-1, 8)
    assert ra.shape == rx.shape
    diff = np.argwhere(ra != rx)
    assert diff.size and set(diff[:, 1].tolist()) == {0}      # only handler ids differ
    fa = jit.records_fingerprint(jit.program_records(p_add, default_leafgen(p_add), 1, full=True)[0])
    fx = jit.records_fingerprint(jit.program_records(p_xor, default_leafgen(p_xor), 1, full=True)[0])
    assert fa != fx


def test_jit_image_entries_point_at_each_program():
    """compile_batch links chunk objects and the table: entry i (relative
    to mg_jit_table) is the first instruction of program i, and its
    fingerprint is that of program i's records."""
    items = []
    for d in (1, 2, 3, 4, 5):
        roots, _ = make_dag(d, SEED)
        p = compile_constraints(roots)
        items.append((p, default_leafgen(p), d))
    image = jit.compile_batch(items, chunk=2)
    with open("/tmp/_mg_jit_test.hsaco", "wb") as fh:
        fh.write(image)
    syms = subprocess.run([jit.LLVM_BIN + "/llvm-readelf", "-s", "/tmp/_mg_jit_test.hsaco"],
                          capture_output=True, text=True, check=True).stdout
    tab = int(re.search(r"([0-9a-f]+)\s+96 OBJECT\s+GLOBAL\s+\w+\s+\d+ mg_jit_table", syms).group(1), 16)
    data = subprocess.run([jit.LLVM_BIN + "/llvm-objdump", "-s", "-j", ".data",
                           "/tmp/_mg_jit_test.hsaco"], capture_output=True, text=True,
                          check=True).stdout
    words = {}
    for line in data.splitlines():
        m = re.match(r"\s*([0-9a-f]+)\s+((?:[0-9a-f]{8}\s?){1,4})", line)
        if m:
            base = int(m.group(1), 16)
            for k, wd in enumerate(m.group(2).split()):
                words[base + 4 * k] = int.from_bytes(bytes.fromhex(wd), "little")
    dis = subprocess.run([jit.LLVM_BIN + "/llvm-objdump", "-d", "/tmp/_mg_jit_test.hsaco"],
                         capture_output=True, text=True, check=True).stdout
    at = {}
    for line in dis.splitlines():
        m = re.search(r"^\s+(\S+).*//\s*([0-9A-F]+):", line)
        if m:
            at[int(m.group(2), 16)] = m.group(1)
    assert words[tab] | words[tab + 4] << 32 == jit.JIT_MAGIC
    assert words[tab + 8] | words[tab + 12] << 32 == int(jit.G.digest()[:16], 16)
    for i, (p, g, s) in enumerate(items):
        row = tab + 16 * (i + 1)
        rel = words[row] | words[row + 4] << 32
        rel -= 1 << 64 if rel >> 63 else 0
        assert rel < 0
        fp = words[row + 8] | words[row + 12] << 32
        full, _ = jit.program_records(p, g, s, full=True)
        assert fp == jit.records_fingerprint(full)
        text = jit.program_asm(p, g, s, "x", tag="p%d" % i)
        first = next(l.split()[0] for l in text[1:] if l.strip() and not l.strip().endswith(":"))
        assert at[tab + rel].startswith(first), (i, at[tab + rel], first)


def test_unsupported_program_stays_on_the_interpreter(monkeypatch):
    """A program the specialiser rejects gets a zero table row (mg_jit_attach
    leaves its descriptor on the interpreter); the others are compiled."""
    items = []
    for d in (1, 2, 3):
        roots, _ = make_dag(d, SEED)
        p = compile_constraints(roots)
        items.append((p, default_leafgen(p), d))
    real = jit.program_asm

    def flaky(p, *a, **k):
        if p is items[1][0]:
            raise jit.JitUnsupported("test")
        return real(p, *a, **k)
    monkeypatch.setattr(jit, "program_asm", flaky)
    fps = []
    text = jit.chunk_asm(items, 0, fps=fps)
    assert fps[1] is None and fps[0] is not None and fps[2] is not None
    assert "mg_jp1:" not in text and "mg_jp0:" in text and "mg_jp2:" in text
    table = jit.table_asm(fps)
    assert "\t.quad 0\n\t.quad 0\n" in table and "mg_jp1" not in table


def _program_digests(order):
    """(worker, spawned fresh) compile the corpus DAGs in ``order``; digest
    of each program's code, constants and record fingerprint."""
    import hashlib
    import bench
    out = {}
    for d in order:
        p = bench.compile_unit(("c2", d))[1]
        full, _ = jit.program_records(p, default_leafgen(p), d, full=True)
        out[d] = (hashlib.sha1(p.code.tobytes() + p.consts.tobytes()).hexdigest(),
                  jit.records_fingerprint(full))
    return out


def test_corpus_programs_do_not_depend_on_build_history():
    """A corpus DAG compiles to the same program whatever its process built
    before (corpus.make_dag builds in a fresh hash-consing scope): the
    compiled-program image one process builds (bench.py --jit-build-only,
    chunk workers) must fit the programs another process loads —
    mg_jit_attach compares their record fingerprints, and refused a cached
    image before this held (constants shared with DAGs built earlier carried
    older ids and moved in the schedule)."""
    import multiprocessing as mp
    ids = list(range(40))
    orders = [ids, ids[::-1]]
    with mp.get_context("spawn").Pool(2) as pool:
        a, b = pool.map(_program_digests, orders)
    assert a == b


def test_branch_materializes_only_what_its_target_reads():
    """jit.specialize: a derived scalar is written to its register before a
    branch only when the code from the branch target may read it; on the
    fall-through path it stays a literal."""
    from mythril_amd.jit import specialize
    b = jit.BANK0
    lines = [
        "    s_and_b32 s80, s%d, 0xff" % b,          # derived: s80 = rec[0] & 0xff
        "    s_add_u32 s81, s%d, 1" % (b + 1),       # derived: s81 = rec[1] + 1
        "    s_cmp_eq_u32 s82, 0",
        "    s_cbranch_scc1 .Ltgt%=",
        "    s_cmp_lt_u32 s83, s80",                 # fall-through reads s80 only
        "    s_branch .Ldone%=",
        ".Ltgt%=:",
        "    s_add_u32 s84, s81, s83",               # the target reads s81 only
        ".Ldone%=:",
        "    s_nop 0",
    ]
    rec = [0x1234, 41, 0, 0, 0, 0, 0, 0]
    hot, cold, _ = specialize(lines, rec, "t")
    text = "\n".join(hot + cold)
    before = text.split("s_cbranch_scc1")[0]
    assert "s_mov_b32 s81, 0x2a" in before          # the target's read, materialized
    assert "s_mov_b32 s80" not in text              # never materialized ...
    assert "s_cmp_lt_u32 s83, 52" in text           # ... the compare takes it inline


def test_code_skipped_by_a_folded_branch_is_inert():
    """after a branch folded as taken, the skipped code up to the
    target emits nothing — a dynamic GPR index, a @@HALT or a @@CALL in it
    neither raises JitUnsupported nor emits instructions or changes the index
    state the target sees."""
    from mythril_amd.jit import specialize
    b = jit.BANK0
    lines = [
        "    s_cmp_eq_u32 s%d, 7" % b,                # rec[0] == 7: folds taken
        "    s_cbranch_scc1 .Ltgt%=",
        "    s_set_gpr_idx_on s90, gpr_idx(SRC0)",     # s90 unknown: dynamic index
        "    v_mov_b32 v0, v8",
        "    s_set_gpr_idx_off",
        "@@CALL DIV 3",
        "@@HALT",
        ".Ltgt%=:",
        "    v_mov_b32 v1, v2",
    ]
    rec = [7, 0, 0, 0, 0, 0, 0, 0]
    hot, cold, call = specialize(lines, rec, "t")
    text = "\n".join(hot + cold)
    assert call is None
    assert "s_setpc" not in text and "s_swappc" not in text and "gpr_idx" not in text
    assert "v_mov_b32 v1, v2" in text and "v_mov_b32 v0" not in text


def test_layout_switch_does_not_reuse_a_dropped_template_analysis():
    """Template analyses (branch targets, reach sets, record fields) are
    memoised by the template list's id(); a layout switch drops the
    templates and a new list may reuse an old id, so a memo hit must be the
    very list (round 6: a stale entry made a regenerated template's labels
    look unreached)."""
    from mythril_amd import asmgen as G
    x = [".Lfoo_%=:", "    s_branch .Lfoo_%="]
    assert jit._branch_targets(x) == frozenset({".Lfoo_%="})
    key = id(x)
    y = [".Lbar_%=:", "    s_branch .Lbar_%="]
    jit._TARGETS[id(y)] = jit._TARGETS.pop(key)   # as if y had reused x's id
    assert jit._branch_targets(y) == frozenset({".Lbar_%="})
    with G.layout(11):
        jit.template("MUL", 0)
    t16 = jit.template("MUL", 0)
    assert jit._branch_targets(t16) == jit._branch_targets(list(t16))
