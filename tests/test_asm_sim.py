"""CPU parity of the hand-written gfx950 assembly interpreter (the product's
hot kernel) through an instruction-level simulator of its exact text
(tests/asm_sim.py) and the library's own IR -> record translator
(mg_translate, host-only).  Every probed node and root bit is compared with
the oracle (oracle/smtlib_ref.py, oracle/gen_ref.py); the same cases run on
the MI355X in test_gpu_parity.py."""

import collections
import random

import numpy as np
import pytest

import asm_sim
import dag_cases
from evm_mini import lower_program
from mythril_amd import asmgen
from mythril_amd.assign import Assignment as PA, pack, unpack
from mythril_amd.corpus import make_dag
from mythril_amd.engine import default_leafgen, limbs_to_int
from mythril_amd.ir import compile_constraints
from mythril_amd.smt import node as N
from oracle import gen_ref
from oracle import smtlib_ref as R
from test_gpu_parity import flat_expected
from test_oracle_golden import load, oracle_eval

CASES = dag_cases.named_cases()
SEED = 0x6D797468


def test_handler_table_is_complete():
    _, table = asm_sim.body_and_table()
    assert len(table) == asmgen.NUM_HANDLERS and min(table) > 0
    canon = {asmgen.canonical(h) for h in range(asmgen.NUM_HANDLERS)}
    assert len(set(table)) == len(canon)          # one body per implemented variant
    for h in range(asmgen.NUM_HANDLERS):
        assert table[h] == table[asmgen.canonical(h)]


def test_generated_text_has_no_scalar_stores():
    text = "\n".join(asmgen.generate())
    for bad in ("s_store", "s_buffer_store", "s_scratch_store", "s_dcache", "s_atomic"):
        assert bad not in text


def _probe_check(prog, probes, asgs, pr, root, constraints):
    for a, asg in enumerate(asgs):
        want = flat_expected(probes, R.evaluate(list(probes), asg))
        got = [limbs_to_int(pr[k, :, a]) for k in range(prog.n_probes)]
        assert got == want, (a, [(i, hex(g), hex(w)) for i, (g, w) in
                                 enumerate(zip(got, want)) if g != w][:4])
        assert bool(root[a]) == bool(R.eval_constraints(constraints, asg)), a


@pytest.mark.parametrize("name", sorted(CASES))
def test_case_parity_sim(name):
    constraints, probes, gen, tables = CASES[name]
    prog = compile_constraints(constraints, probes, table_sizes=tables)
    rng = random.Random(2000 + len(name))
    asgs = [gen(rng) for _ in range(64)]
    soa = pack(prog, [PA(a.vars, a.arrays, a.funcs) for a in asgs])
    root, pr, _, _ = asm_sim.simulate(prog, soa)
    _probe_check(prog, probes, asgs, pr, root, constraints)


def test_division_edges_with_reciprocal_noise():
    """Every division operator on edge values, with v_rcp_f64 perturbed by
    up to 1e-7 relative (the integer correction must absorb it)."""
    x, y = N.bv_var("x", 256), N.bv_var("y", 256)
    probes = [N.bv_op(op, x, y) for op in ("bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod")]
    prog = compile_constraints([], probes)
    rng = random.Random(3)
    edges = [0, 1, 2, 3, (1 << 31), (1 << 32) - 1, 1 << 32, (1 << 64) - 1, 1 << 255,
             (1 << 256) - 1, (1 << 255) - 1, (1 << 128) + 1, 0xFFFFFFFF00000000]
    for rep in range(3):
        asgs = [PA(vars={"x": rng.choice(edges + [rng.getrandbits(rng.choice((32, 64, 200, 256)))]),
                         "y": rng.choice(edges + [rng.getrandbits(rng.choice((31, 33, 64, 130, 256)))])})
                for _ in range(64)]
        root, pr, _, _ = asm_sim.simulate(prog, pack(prog, asgs), rcp_noise=1e-7)
        for a, asg in enumerate(asgs):
            want = R.evaluate(probes, R.Assignment(asg.vars))
            got = [limbs_to_int(pr[k, :, a]) for k in range(len(probes))]
            assert got == want, (rep, a, hex(asg.vars["x"]), hex(asg.vars["y"]))


@pytest.mark.parametrize("rep", range(3))
def test_division_one_limb_waves(rep):
    """Waves whose every divisor magnitude fits 32 bits take the short
    division (asmgen._udivrem_short): zero divisors, 1, 2^31, 2^32 - 1,
    small negative divisors for the signed operators, dividends of every
    length, reciprocal perturbed."""
    x, y = N.bv_var("x", 256), N.bv_var("y", 256)
    probes = [N.bv_op(op, x, y) for op in ("bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod")]
    prog = compile_constraints([], probes)
    rng = random.Random(40 + rep)
    small = [0, 1, 2, 3, 7, 1 << 31, (1 << 31) + 1, (1 << 32) - 1, 0x10001, 10 ** 9]
    asgs = []
    for _ in range(64):
        d = rng.choice(small + [rng.getrandbits(rng.choice((8, 20, 31, 32)))])
        if rep == 2 and rng.random() < 0.5:
            d = (1 << 256) - d if d else 0                   # small negative divisors
        xv = rng.choice([0, 1, (1 << 256) - 1, 1 << 255, rng.getrandbits(256),
                         rng.getrandbits(rng.randrange(1, 256))])
        asgs.append(PA(vars={"x": xv, "y": d}))
    # (rep 2: for the unsigned operators such a divisor is wide: the wave
    # takes the generic path for them; the signed ones see |d| < 2^32)
    root, pr, _, _ = asm_sim.simulate(prog, pack(prog, asgs), rcp_noise=1e-7)
    for a, asg in enumerate(asgs):
        want = R.evaluate(probes, R.Assignment(asg.vars))
        got = [limbs_to_int(pr[k, :, a]) for k in range(len(probes))]
        assert got == want, (rep, a, hex(asg.vars["x"]), hex(asg.vars["y"]))


# (d, u1, u0) where the Moller-Granlund 2-by-1 step (r:u) = (u1:u0) needs
# its second, "unlikely" correction (r' >= d): found by brute force over the
# algorithm restated in Python (round 5 moved that correction behind a branch)
MG_SECOND_CORRECTION = [(2322326124, 2251310039, 4214312352), (2267272354, 2057016691, 4168275397),
                        (2996589211, 2755454550, 4001446354)]


def test_short_division_second_correction():
    """The one-limb short division's rare second quotient correction: lanes
    that need it, lanes that do not, in one wave, at several digit positions
    (a normalised divisor, so the step sees (u1:u0) itself, and shifted
    divisors, which move it)."""
    x, y = N.bv_var("x", 256), N.bv_var("y", 256)
    probes = [N.bv_op("bvudiv", x, y), N.bv_op("bvurem", x, y)]
    prog = compile_constraints([], probes)
    rng = random.Random(7)
    asgs = []
    for lane in range(64):
        d, u1, u0 = MG_SECOND_CORRECTION[lane % 3]
        pos = rng.randrange(7)
        xv = ((u1 << 32) | u0) << (32 * pos) | rng.getrandbits(32 * pos)
        if lane % 5 == 4:
            xv, d = rng.getrandbits(256), rng.getrandbits(32) | 1
        asgs.append(PA(vars={"x": xv, "y": d}))
    root, pr, _, _ = asm_sim.simulate(prog, pack(prog, asgs))
    for a, asg in enumerate(asgs):
        want = R.evaluate(probes, R.Assignment(asg.vars))
        got = [limbs_to_int(pr[k, :, a]) for k in range(len(probes))]
        assert got == want, (a, hex(asg.vars["x"]), hex(asg.vars["y"]))


@pytest.mark.parametrize("rep", range(3))
def test_division_two_limb_waves(rep):
    """Waves whose every divisor magnitude fits 64 bits and some lane's does
    not fit 32 take the 3-by-2 short division (asmgen._udivrem_short2):
    divisors of 33..64 bits mixed with one-limb and zero divisors (those
    lanes move up a limb), 2^63, 2^64 - 1, signed operators with small
    negative divisors, dividends of every length, reciprocal perturbed."""
    x, y = N.bv_var("x", 256), N.bv_var("y", 256)
    probes = [N.bv_op(op, x, y) for op in ("bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod")]
    prog = compile_constraints([], probes)
    rng = random.Random(90 + rep)
    edge = [0, 1, 3, (1 << 32) - 1, 1 << 32, (1 << 32) + 1, (1 << 63), (1 << 64) - 1,
            (1 << 63) + 1, 0xFFFFFFFF00000000, 10 ** 18]
    asgs = []
    for lane in range(64):
        d = rng.choice(edge + [rng.getrandbits(rng.choice((33, 40, 63, 64))),
                               rng.getrandbits(rng.choice((8, 31, 32)))])
        if lane == 0:
            d = (1 << 40) + 7                               # every wave has a two-limb divisor
        if rep == 2 and rng.random() < 0.5 and d:
            d = (1 << 256) - d                              # negative: |d| fits 64 bits
        xv = rng.choice([0, 1, (1 << 256) - 1, 1 << 255, rng.getrandbits(256),
                         rng.getrandbits(rng.randrange(1, 256)), rng.getrandbits(64)])
        asgs.append(PA(vars={"x": xv, "y": d}))
    root, pr, _, _ = asm_sim.simulate(prog, pack(prog, asgs), rcp_noise=1e-7)
    for a, asg in enumerate(asgs):
        want = R.evaluate(probes, R.Assignment(asg.vars))
        got = [limbs_to_int(pr[k, :, a]) for k in range(len(probes))]
        assert got == want, (rep, a, hex(asg.vars["x"]), hex(asg.vars["y"]))


@pytest.mark.parametrize("w", [256, 64, 8])
def test_division_by_zero_waves(w):
    """A wave whose every divisor is zero skips the division (quotient and
    remainder 0, then SMT-LIB's x/0 rules) — every operator, dividends of
    both signs, at several widths."""
    x, y = N.bv_var("x", w), N.bv_var("y", w)
    probes = [N.bv_op(op, x, y) for op in ("bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod")]
    prog = compile_constraints([], probes)
    rng = random.Random(w)
    M = (1 << w) - 1
    asgs = [PA(vars={"x": rng.choice([0, 1, M, 1 << (w - 1), rng.getrandbits(w)]), "y": 0})
            for _ in range(64)]
    root, pr, _, _ = asm_sim.simulate(prog, pack(prog, asgs))
    for a, asg in enumerate(asgs):
        want = R.evaluate(probes, R.Assignment(asg.vars))
        got = [limbs_to_int(pr[k, :, a]) for k in range(len(probes))]
        assert got == want, (w, a, hex(asg.vars["x"]))


@pytest.mark.parametrize("mode", ["all_large", "one_small", "w160"])
def test_umulno_overflow_waves(mode):
    """bvumul_noovfl: a W = 256 wave whose operands are all >= 2^128 answers
    "overflow" without bit lengths (asmgen.h_umulno's wave exit); a lane with a small
    operand, or a narrower width, takes the bit-length path."""
    w = 160 if mode == "w160" else 256
    x, y = N.bv_var("x", w), N.bv_var("y", w)
    probes = [N.ite(N.bv_cmp("bvumul_noovfl", x, y), x, y),
              N.ite(N.bv_cmp("bvumul_noovfl", y, x), y, x)]
    prog = compile_constraints([], probes)
    rng = random.Random(len(mode))
    half = w // 2
    asgs = []
    for lane in range(64):
        xv = rng.getrandbits(w - half) << half | rng.getrandbits(half) | 1 << (w - 1 - rng.randrange(w - half))
        yv = rng.getrandbits(w - half) << half | 1 << half
        if mode == "one_small" and lane == 37:
            yv = rng.getrandbits(100)
        asgs.append(PA(vars={"x": xv & ((1 << w) - 1), "y": yv & ((1 << w) - 1)}))
    root, pr, _, _ = asm_sim.simulate(prog, pack(prog, asgs))
    for a, asg in enumerate(asgs):
        want = R.evaluate(probes, R.Assignment(asg.vars))
        got = [limbs_to_int(pr[k, :, a]) for k in range(len(probes))]
        assert got == want, (mode, a)


def _div3by2_unlikely(rng):
    """(d, r, u0) with d normalised to 64 bits and r < d where the 3-by-2
    step needs its rare final correction (a restatement of Moller-Granlund's
    Algorithms 5 and 6 over 32-bit words, searched at random)."""
    B, M = 1 << 32, (1 << 32) - 1
    while True:
        d = rng.getrandbits(64) | 1 << 63
        d1, d0 = d >> 32, d & M
        v = (B ** 3 - 1) // d - B
        r = rng.randrange(d)
        u0 = rng.getrandbits(32)
        u2, u1 = r >> 32, r & M
        q = v * u2 + (u2 << 32 | u1)
        q1, q0 = (q >> 32) & M, q & M
        r1 = (u1 - q1 * d1) & M
        rr = ((r1 << 32 | u0) - d0 * q1 - d) % (B * B)
        if rr >> 32 >= q0:
            rr = (rr + d) % (B * B)
        if rr >= d:
            return d, r, u0


def test_two_limb_division_final_correction():
    """Lanes whose 3-by-2 step needs the final ("unlikely") correction, at
    several digit positions, next to lanes that do not."""
    x, y = N.bv_var("x", 256), N.bv_var("y", 256)
    probes = [N.bv_op("bvudiv", x, y), N.bv_op("bvurem", x, y)]
    prog = compile_constraints([], probes)
    rng = random.Random(11)
    cases = [_div3by2_unlikely(rng) for _ in range(4)]
    asgs = []
    for lane in range(64):
        d, r, u0 = cases[lane % 4]
        pos = rng.randrange(6)
        xv = (r << 32 | u0) << (32 * pos) | rng.getrandbits(32 * pos)
        if lane % 7 == 6:
            xv, d = rng.getrandbits(256), rng.getrandbits(64) | 1
        asgs.append(PA(vars={"x": xv, "y": d}))
    root, pr, _, _ = asm_sim.simulate(prog, pack(prog, asgs))
    for a, asg in enumerate(asgs):
        want = R.evaluate(probes, R.Assignment(asg.vars))
        got = [limbs_to_int(pr[k, :, a]) for k in range(len(probes))]
        assert got == want, (a, hex(asg.vars["x"]), hex(asg.vars["y"]))


@pytest.mark.parametrize("small", ["y", "x", "both", "none"])
def test_mul_short_operand_waves(small):
    """MUL waves whose operands are below 2^64 in every lane (either side,
    both, or all but one lane) against the oracle at several widths (round
    4 measured a two-row product for such waves and dropped it)."""
    rng = random.Random(len(small))
    for w in (256, 160, 64):
        x, y = N.bv_var("x", w), N.bv_var("y", w)
        probes = [N.bv_op("bvmul", x, y), N.bv_op("bvmul", y, x)]
        prog = compile_constraints([], probes)
        M = (1 << w) - 1
        asgs = []
        for lane in range(64):
            xv, yv = rng.getrandbits(w), rng.getrandbits(w)
            if small in ("x", "both"):
                xv = rng.choice([0, 1, (1 << 64) - 1, rng.getrandbits(64), rng.getrandbits(33)])
            if small in ("y", "both"):
                yv = rng.choice([0, 1, (1 << 64) - 1, rng.getrandbits(64), rng.getrandbits(32)])
            if small == "none" and lane == 17:
                xv, yv = M, M
            elif small == "none":
                yv = rng.getrandbits(60)
            asgs.append(PA(vars={"x": xv & M, "y": yv & M}))
        root, pr, _, _ = asm_sim.simulate(prog, pack(prog, asgs))
        for a, asg in enumerate(asgs):
            want = R.evaluate(probes, R.Assignment(asg.vars))
            got = [limbs_to_int(pr[k, :, a]) for k in range(len(probes))]
            assert got == want, (small, w, a)


@pytest.mark.parametrize("spans", [(1, 33, 64), (65, 100, 128), (1, 64, 128), (1, 64, 256)])
def test_division_short_divisor_chains(spans):
    """Waves whose divisors span few digits (any position, after
    normalisation: the multiply-subtract enters at digit 6 or 4 when every
    lane with a nonzero quotient digit allows it), mixed with zero-quotient
    lanes of wide divisors."""
    x, y = N.bv_var("x", 256), N.bv_var("y", 256)
    probes = [N.bv_op(op, x, y) for op in ("bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod")]
    prog = compile_constraints([], probes)
    rng = random.Random(sum(spans))
    for rep in range(2):
        asgs = []
        for _ in range(64):
            span = rng.choice(spans)
            yv = (rng.getrandbits(span) | 1 << (span - 1)) << rng.randrange(0, 257 - span)
            xv = rng.getrandbits(256) if rng.random() < 0.8 else rng.getrandbits(rng.randrange(1, 256))
            asgs.append(PA(vars={"x": xv, "y": yv}))
        root, pr, _, _ = asm_sim.simulate(prog, pack(prog, asgs))
        for a, asg in enumerate(asgs):
            want = R.evaluate(probes, R.Assignment(asg.vars))
            got = [limbs_to_int(pr[k, :, a]) for k in range(len(probes))]
            assert got == want, (rep, a, hex(asg.vars["x"]), hex(asg.vars["y"]))


def _max_qhat_error(x: int, y: int) -> int:
    """Largest (estimate - true digit) of Knuth D's two-digit quotient
    estimate over the digits of x / y (32-bit digits, normalised)."""
    B = 1 << 32
    sh = 256 - y.bit_length()
    un = [((x << sh) >> (32 * i)) & (B - 1) for i in range(17)]
    V = y << sh
    worst = 0
    for j in range(7, -1, -1):
        window = sum(un[j + i] << (32 * i) for i in range(9))
        q = window // V
        qh = min((un[j + 8] * B + un[j + 7]) // (V >> 224), B - 1)
        worst = max(worst, qh - q)
        r = window - q * V
        for i in range(9):
            un[j + i] = (r >> (32 * i)) & (B - 1)
    return worst


def test_hard_division_case_reaches_double_correction():
    """The division_hard case (run by test_case_parity_sim here and by the
    GPU parity suite) does exercise a quotient estimate two too big, the
    path that takes the second add-back."""
    rng = random.Random(2000 + len("division_hard"))
    errs = [_max_qhat_error(*dag_cases.hard_division_pair(rng)) for _ in range(64)]
    assert max(errs) == 2 and errs.count(2) >= 3


@pytest.mark.parametrize("dag_id,n_lds", [(0, 6), (1, 0), (7, 2), (33, 6)])
def test_corpus_constraints_as_probes_generated(dag_id, n_lds):
    """A corpus DAG with every constraint probed (so each lane checks ~half
    true bits), candidates from the device generator, spills split between
    LDS and scratch as n_lds says."""
    roots, _ = make_dag(dag_id, SEED)
    prog = compile_constraints([], roots)
    lg = default_leafgen(prog)
    first = 777 * dag_id
    _, pr, lout, _ = asm_sim.simulate(prog, gen=(SEED, dag_id, first, lg), n_lds=n_lds,
                                      want_leaves=True)
    pool = prog.const_values
    for lane in range(64):
        lv = [gen_ref.gen_leaf(SEED, dag_id, li, first + lane, l.width, pool)
              for li, l in enumerate(prog.leaves)]
        assert [limbs_to_int(lout[li, :, lane]) for li in range(len(prog.leaves))] == lv
        asg = unpack(prog, lout[:, :, lane])
        want = R.evaluate(list(roots), R.Assignment(asg.vars, asg.arrays, asg.funcs))
        got = [int(pr[k, 0, lane]) for k in range(len(roots))]
        assert got == [int(w) for w in want], lane


def test_vmtests_sim():
    checked = 0
    for t in load("vmtests.json")[::3]:
        vars_, stores, divergent = lower_program(t["code"], oracle_eval)
        if divergent or not stores:
            continue
        probes = [v.raw for _, v in stores] + [k.raw for k, _ in stores]
        prog = compile_constraints([], probes)
        _, pr, _, _ = asm_sim.simulate(prog, pack(prog, [PA(vars=vars_)] * 64))
        n = len(stores)
        storage = {limbs_to_int(pr[n + i, :, 0]): limbs_to_int(pr[i, :, 0]) for i in range(n)}
        storage = {k: v for k, v in storage.items() if v}
        assert storage == {int(k, 16): int(v, 16) for k, v in t["storage"].items()}, t["name"]
        checked += 1
    assert checked >= 40


def test_inactive_lanes_do_not_store():
    x = N.bv_var("x", 256)
    prog = compile_constraints([], [N.bv_op("bvadd", x, x)])
    asgs = [PA(vars={"x": i + 1}) for i in range(64)]
    active = (1 << 40) - 1
    _, pr, _, _ = asm_sim.simulate(prog, pack(prog, asgs), active=active)
    for a in range(64):
        assert limbs_to_int(pr[0, :, a]) == (2 * (a + 1) if a < 40 else 0)


def _record_handlers(prog):
    """(family, variant) of every translated record of prog."""
    _, table = asm_sim.body_and_table()
    off2 = {}
    for h, off in enumerate(table):
        bank, var, aop = h % 2, (h // 2) % asmgen.NVAR, h // (2 * asmgen.NVAR)
        off2.setdefault(off, (asmgen.AOPS[aop], var))
    rec, _ = asm_sim.translate(prog, 6)
    return [off2.get(int(r[0]), ("PAD", 0)) for r in rec.reshape(-1, 8)]   # + zeroed pad


def test_nw_variant_only_for_dead_root_conjuncts():
    """A ROOT-fused compare nobody reads later takes the no-write variant
    (only the root is updated); one whose value is read again (here by an
    ITE) keeps writing its slot.  Both roots stay right (simulated)."""
    x, y, z = N.bv_var("x", 256), N.bv_var("y", 256), N.bv_var("z", 256)
    live = N.bv_cmp("bvule", x, y)                  # also the ITE's condition
    dead = N.bv_cmp("bvult", z, x)                  # a root only
    pick = N.ite(live, z, y)
    roots = [live, dead, N.distinct(pick, N.bv_num(7, 256))]
    prog = compile_constraints(roots)
    fams = _record_handlers(prog)
    ule = [var for f, var in fams if f == "ULE"]
    ult = [var for f, var in fams if f == "ULT"]
    assert ule and not any(var & asmgen.V_NW for var in ule)
    assert ult and all(var & asmgen.V_NW for var in ult)
    rng = random.Random(5)
    asgs = [PA(vars={k: rng.choice([0, 1, 7, (1 << 256) - 1, rng.getrandbits(256)])
                     for k in ("x", "y", "z")}) for _ in range(64)]
    root, _, _, _ = asm_sim.simulate(prog, pack(prog, asgs))
    for a, asg in enumerate(asgs):
        assert bool(root[a]) == bool(R.eval_constraints(roots, asg)), a


def test_index_mode_text_invariants():
    """GPR-index mode is state, not brackets: an off never
    directly precedes an on (s_set_gpr_idx_on sets index and mode in any
    state), and in every handler the first instruction that touches VGPRs,
    or the first branch, comes after the handler set the mode itself (a
    handler may be entered with the mode left on by the previous one)."""
    lines = [l.strip() for l in asmgen.generate()]
    for a, b in zip(lines, lines[1:]):
        assert not (a == "s_set_gpr_idx_off" and b.startswith("s_set_gpr_idx_on")), (a, b)
    for i, t in enumerate(lines):
        if not (t.startswith(".Lh") and t.endswith(":")):
            continue
        for u in lines[i + 1:]:
            op = u.split(None, 1)[0] if u else ""
            if op.startswith("s_set_gpr_idx_on") or op == "s_set_gpr_idx_off" or \
                    op == "s_setpc_b64" or u.startswith("s_branch .Lbody_"):
                break                 # (a heavy body sets the mode itself)
            assert not (op.startswith("v_") or op.startswith("ds_") or
                        op.startswith("global_") or op.startswith("scratch_") or
                        op.startswith("s_cbranch") or op == "s_branch"), (t, u)


@pytest.mark.parametrize("workload,unit,n_lds,jit", [("c3", 16, 6, False), ("c3", 16, 6, True),
                                                     ("c3", 41, 2, True), ("c5", 46, 6, True),
                                                     ("c4", 9, 6, False)])
def test_spill_placement_stand_in_units(workload, unit, n_lds, jit):
    """Spill placement (mg_host.cpp place_spills, round 5): one-limb values
    packed eight to an LDS region, 256-bit values in whole regions, the rest
    in re-coloured scratch positions, spills nobody reloads dropped.  A bench
    unit of the spill-heaviest stand-in workloads, interpreted and compiled,
    must give the oracle's root bit on every lane, and its records must use
    the narrow LDS and scratch variants."""
    import bench
    from mythril_amd import asmgen
    from mythril_amd.engine import translate_records
    _, prog, _, _ = bench.compile_unit((workload, unit))
    rec, _ = translate_records(prog, n_lds)
    fams = collections.Counter()
    for h in rec.reshape(-1, 8)[:, 0]:
        name, var = asmgen.AOPS[int(h) // (2 * asmgen.NVAR)], (int(h) // 2) % asmgen.NVAR
        fams[(name, bool(var & asmgen.V_NARROW) if name in (
            "SPILL_LDS", "RELOAD_LDS", "SPILL_SCR", "RELOADD") else False)] += 1
    assert fams[("SPILL_LDS", True)] and fams[("RELOAD_LDS", True)] and fams[("SPILL_SCR", False)]
    lg = default_leafgen(prog)
    first = 64 * 1001 + unit
    root, _, lout, _ = asm_sim.simulate(prog, gen=(SEED, unit, first, lg), n_lds=n_lds,
                                        want_leaves=True, jit=jit)
    roots = bench.workload_roots(workload, unit)
    for lane in range(64):
        asg = unpack(prog, lout[:, :, lane])
        want = R.eval_constraints(list(roots), R.Assignment(asg.vars, asg.arrays, asg.funcs))
        assert bool(root[lane]) == bool(want), lane


@pytest.mark.parametrize("jit", [False, True])
def test_dirty_one_limb_value_never_reaches_eqsel(jit):
    """a one-limb result left dirty (limbs 1..7 stale,
    the DC handler writes limb 0 only) is safe only for limb-0 readers.  A
    w <= 32 ITE right after a wide EQ on its condition is fused into EQSEL,
    which copies all eight limbs of its value operands and marks the result
    clean — so a dirty value operand must not be left dirty.  Hand-written
    IR: slot 4 holds a wide leaf, EXTRACT w=8 overwrites it, EQ(w=256) +
    ITE(w=8) select it, and the ITE result is read at full width (OUT and a
    256-bit ADD)."""
    from mythril_amd import irdefs as I
    x, y, k, z = (N.bv_var(n, 256) for n in ("x", "y", "k", "z"))
    v = N.bv_var("v", 8)
    base = compile_constraints([], [x, y, k, z, v, x])
    li = {l.name: i for i, l in enumerate(base.leaves)}
    code = [
        (I.w0(I.LEAF, 256), I.w1(0), li["x"]),
        (I.w0(I.LEAF, 256), I.w1(1), li["y"]),
        (I.w0(I.LEAF, 256), I.w1(2), li["k"]),
        (I.w0(I.LEAF, 8), I.w1(3), li["v"]),
        (I.w0(I.LEAF, 256), I.w1(4), li["z"]),               # slot 4: a wide value
        (I.w0(I.EXTRACT, 8), I.w1(4, 0), 0),                  # x[7:0] into slot 4
        (I.w0(I.EQ, 256), I.w1(5, 1, 2), 0),
        (I.w0(I.ITE, 8), I.w1(6, 4, 3, 5), 0),                # EQSEL candidate
        (I.w0(I.OUT, 8), I.w1(0, 6), 0),
        (I.w0(I.ADD, 256), I.w1(7, 6, 6), 0),
        (I.w0(I.OUT, 256), I.w1(0, 7), 1),
    ]
    prog = base
    prog.code = np.array([[a, b, c, 0] for a, b, c in code], dtype=np.uint32)
    prog.n_probes = 2
    fams = [f for f, _ in _record_handlers(prog)]
    assert "EQSEL" in fams and "ITE" not in fams         # the fused shape is exercised
    rng = random.Random(11)
    asgs = []
    for lane in range(64):
        yy = rng.getrandbits(256)
        asgs.append(PA(vars={"x": rng.getrandbits(256), "y": yy,
                             "k": yy if lane % 2 else rng.getrandbits(256),
                             "z": (1 << 256) - 1 - lane, "v": rng.getrandbits(8)}))
    _, pr, _, _ = asm_sim.simulate(prog, pack(prog, asgs), jit=jit)
    for a, asg in enumerate(asgs):
        vv = asg.vars
        sel = (vv["x"] & 0xFF) if vv["y"] == vv["k"] else vv["v"]
        assert limbs_to_int(pr[0, :, a]) == sel, (a, hex(limbs_to_int(pr[0, :, a])))
        assert limbs_to_int(pr[1, :, a]) == 2 * sel, a
