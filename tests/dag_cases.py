"""Test infrastructure: named constraint sets with probes and assignment
generators, shared by the CPU compiler tests (tests/test_compiler.py, through
tests/ir_sim.py) and the GPU parity tests (tests/test_gpu_parity.py).

Every probe is a DAG node whose value the engine writes out per assignment,
so a case checks every intermediate value bit-exactly, not only the root.
"""

import random

from mythril_amd.smt import node as N
from oracle.smtlib_ref import Assignment

WIDTHS = (1, 7, 8, 31, 32, 33, 63, 64, 65, 127, 128, 160, 200, 255, 256)


def edge_value(rng: random.Random, w: int) -> int:
    m = (1 << w) - 1
    k = rng.randrange(10)
    if k == 0:
        return 0
    if k == 1:
        return 1
    if k == 2:
        return m
    if k == 3:
        return 1 << (w - 1)
    if k == 4:
        return (1 << (w - 1)) - 1
    if k == 5:
        return rng.getrandbits(min(w, 64))
    if k == 6:
        b = rng.randrange(w)
        return ((1 << b) + rng.choice((-1, 0, 1))) & m
    return rng.getrandbits(w)


BIN = ["bvadd", "bvsub", "bvmul", "bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod",
       "bvand", "bvor", "bvxor", "bvshl", "bvlshr", "bvashr"]
CMP = ["bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle", "bvsgt", "bvsge", "bvumul_noovfl"]


def all_ops_case(w: int):
    """Every bit-vector operator at width w on two variables (and a small
    shift amount), every node probed."""
    x, y = N.bv_var("x%d" % w, w), N.bv_var("y%d" % w, w)
    probes = []
    for op in BIN:
        probes.append(N.bv_op(op, x, y))
    probes += [N.bv_op("bvneg", x), N.bv_op("bvnot", y)]
    bools = [N.bv_cmp(op, x, y) for op in CMP] + [N.eq(x, y), N.distinct(x, y)]
    probes += [N.ite(b, x, y) for b in bools]
    if w > 1:
        lo = w // 3
        probes.append(N.extract(w - 1, lo, x))
        probes.append(N.zero_extend(256 - w, x) if w < 256 else x)
        probes.append(N.sign_extend(256 - w, y) if w < 256 else y)
        probes.append(N.concat(N.extract(w // 2, 0, x), N.extract(w - 1, w // 2 + 1, y))
                      if w > 2 else x)
    if w <= 128:
        probes.append(N.concat(x, y))
    constraints = [N.bool_op("or", bools[0], bools[1])]

    def gen(rng):
        return Assignment(vars={x.params[0]: edge_value(rng, w), y.params[0]: edge_value(rng, w)})
    return constraints, probes, gen


def bool_case():
    a, b, c = N.bool_var("a"), N.bool_var("b"), N.bool_var("c")
    x, y = N.bv_var("bx", 256), N.bv_var("by", 256)
    probes = [N.bool_op("and", a, b, c), N.bool_op("or", a, b, c), N.bool_op("xor", a, b),
              N.bool_op("not", a), N.bool_op("=>", a, b), N.eq(a, b), N.distinct(a, b, c),
              N.ite(a, b, c), N.ite(N.bool_op("xor", a, c), x, y),
              N.distinct(x, y, N.bv_num(3, 256))]
    constraints = [N.bool_op("or", a, N.bool_op("not", b)), N.bool_op("=>", c, a)]

    def gen(rng):
        return Assignment(vars={"a": rng.randrange(2), "b": rng.randrange(2), "c": rng.randrange(2),
                                "bx": edge_value(rng, 256), "by": rng.choice((3, 4, edge_value(rng, 256)))})
    return constraints, probes, gen


def array_case(entries=3):
    """select over store chains, K arrays, free arrays (model tables), and an
    array-valued ite — the shapes of calldata/storage/balance reads."""
    A = N.array_var("A", 256, 256)
    cd = N.array_var("cd", 256, 8)
    i, j, k, v = (N.bv_var(n, 256) for n in ("ai", "aj", "ak", "av"))
    st = N.store(N.store(A, i, v), j, N.bv_op("bvadd", v, N.bv_num(1, 256)))
    kst = N.store(N.const_array(256, N.bv_num(0, 256)), i, v)
    c = N.bv_cmp("bvult", i, j)
    # a zero-extended narrow value stored over a wide one: the lowered store
    # link is an ite whose arms differ in width (C2 DAG 571, round 3)
    nv = N.zero_extend(240, N.extract(79, 64, v))
    st2 = N.store(N.store(A, i, v), j, nv)
    probes = [N.select(A, k), N.select(st, k), N.select(st, i), N.select(st, j),
              N.select(kst, k), N.select(kst, i), N.select(cd, k),
              N.select(N.ite(c, st, kst), k), N.select(st2, i), N.select(st2, k),
              N.ite(c, nv, v)]
    # calldata word as LASER builds it (calldata.py:219-232): concat of 4 bytes
    size = N.bv_var("cdsize", 256)
    parts = []
    for off in range(4):
        idx = N.bv_op("bvadd", k, N.bv_num(off, 256))
        parts.append(N.ite(N.bv_cmp("bvslt", idx, size), N.select(cd, idx), N.bv_num(0, 8)))
    word = N.concat(*parts)
    probes.append(word)
    constraints = [N.eq(N.select(cd, k), N.bv_num(0xA9, 8))]

    def gen(rng):
        keys = [edge_value(rng, 256) for _ in range(entries)]
        ivals = [rng.choice(keys + [edge_value(rng, 256)]) for _ in range(3)]
        tabA = ([(kk, edge_value(rng, 256)) for kk in keys[:rng.randrange(entries + 1)]],
                edge_value(rng, 256))
        base = rng.choice(ivals)
        tabcd = ([((base + o) % (1 << 256), rng.randrange(256)) for o in range(rng.randrange(entries + 1))],
                 rng.randrange(256))
        return Assignment(vars={"ai": ivals[0], "aj": ivals[1], "ak": base,
                                "av": edge_value(rng, 256), "cdsize": rng.choice((0, 2, 4, 100))},
                          arrays={"A": tabA, "cd": tabcd})
    return constraints, probes, gen, {"A": entries, "cd": entries}


def _cd_word(cd, size, off, numerals_first=False, const_base=None):
    """LASER's calldata word (calldata.py:47-54,219-232): 32 bytes
    If(off + i <s size, cd[off + i], 0), high byte first."""
    parts = []
    for i in range(32):
        if const_base is not None:
            idx = N.bv_num((const_base + i) % (1 << 256), 256)
        elif i == 0:
            idx = off
        elif numerals_first:
            idx = N.bv_op("bvadd", N.bv_num(i, 256), off)
        else:
            idx = N.bv_op("bvadd", off, N.bv_num(i, 256))
        parts.append(N.ite(N.bv_cmp("bvslt", idx, size), N.select(cd, idx), N.bv_num(0, 8)))
    return N.concat(*parts)


# offsets around every edge of the word: the signed wrap of off + i at
# 2^255 (u = off ^ 2^255 wraps at 2^256), the unsigned wrap of the index at
# 2^256, zero, and ordinary ABI offsets
CD_OFFSETS = (0, 4, 36, 68, (1 << 255) - 32, (1 << 255) - 31, (1 << 255) - 17, (1 << 255) - 1,
              1 << 255, (1 << 256) - 32, (1 << 256) - 16, (1 << 256) - 1, (1 << 32) - 5,
              ((1 << 32) - 5) | (0x7FFFFFFF << 224) | (((1 << 192) - 1) << 32))


def calldata_word_case(entries=4):
    """Calldata words over a free array read through its model table (the
    fused BCAST / CDWE / CDWX chain, ir.py _calldata_word): symbolic
    offsets (both bvadd operand orders), a constant offset, sizes that
    straddle the word, sizes with the sign bit set, offsets at the signed
    and unsigned wrap points, and table keys that hit the word at random
    bytes, past its ends and more than once (first match wins)."""
    cd = N.array_var("cdw", 256, 8)
    size = N.bv_var("cdw_size", 256)
    o1, o2 = N.bv_var("cdw_o1", 256), N.bv_var("cdw_o2", 256)
    w1 = _cd_word(cd, size, o1)
    w2 = _cd_word(cd, size, o2, numerals_first=True)
    w3 = _cd_word(cd, size, None, const_base=4)
    w4 = _cd_word(cd, size, N.bv_op("bvadd", o1, N.bv_num(4, 256)))
    probes = [w1, w2, w3, w4, N.bv_op("bvxor", w1, w3)]
    constraints = [N.bv_cmp("bvult", w3, w1)]

    def gen(rng):
        offs = [rng.choice(CD_OFFSETS) if rng.randrange(3) else edge_value(rng, 256)
                for _ in range(2)]
        ents = []
        for _ in range(rng.randrange(entries + 1)):
            base = rng.choice(offs + [4, 8])
            key = (base + rng.choice((rng.randrange(-2, 36), rng.randrange(32)))) % (1 << 256)
            ents.append((key, rng.randrange(256)))
        sizes = [0, 1, 4, 35, 36, 40, 67, 68, 100, 1 << 255, (1 << 255) - 1, (1 << 256) - 1]
        k = rng.randrange(4)
        if k == 0:
            sz = rng.choice(sizes)
        elif k == 1:
            sz = (rng.choice(offs) + rng.randrange(-3, 36)) % (1 << 256)
        elif k == 2:
            sz = edge_value(rng, 256)
        else:
            sz = ((1 << 255) - rng.randrange(40)) % (1 << 256)
        return Assignment(vars={"cdw_o1": offs[0], "cdw_o2": offs[1], "cdw_size": sz},
                          arrays={"cdw": (ents, rng.randrange(256))})
    return constraints, probes, gen, {"cdw": entries}


def keccak_uf_case(words: int = 2):
    """The UF-pair shape of keccak_function_manager.py:121-149 on a 512-bit
    (mapping-slot) input: keccak256_512(concat(key, slot)) with the interval /
    mod-64 conditions and the inverse function.  ``words=3``: a 768-bit input
    (concat(key, key2, slot): wider than the 512-bit C oracle build, so it
    runs on the wide one)."""
    bits = 256 * words
    key, slot = N.bv_var("kkey", 256), N.bv_var("kslot", 256)
    data = N.concat(key, slot) if words == 2 else N.concat(N.concat(key, N.bv_var("kkey2", 256)), slot)
    fn = "keccak256_%d" % bits
    f = lambda t: N.apply_uf(fn, bits, 256, t)                   # noqa: E731
    inv = lambda t: N.apply_uf(fn + "-1", 256, bits, t)          # noqa: E731
    h = f(data)
    TOTAL_PARTS = 10 ** 40
    PART = (2 ** 256 - 1) // TOTAL_PARTS
    lo = (TOTAL_PARTS - 34534) * PART
    cond = N.bool_op("and", N.eq(inv(h), data),
                     N.bool_op("or", N.bv_cmp("bvult", N.bv_num(lo, 256), h), N.eq(N.bv_num(lo, 256), h)),
                     N.bv_cmp("bvult", h, N.bv_num(lo + PART, 256)),
                     N.eq(N.bv_op("bvurem", h, N.bv_num(64, 256)), N.bv_num(0, 256)))
    probes = [h, inv(h), N.extract(300, 100, data), N.extract(bits - 1, bits - 256, inv(h)),
              N.zero_extend(256, key)]
    constraints = [cond]

    def gen(rng):
        kv, sv = edge_value(rng, 256), rng.randrange(8)
        vars_ = {"kkey": kv, "kslot": sv}
        d = (kv << 256) | sv
        if words == 3:
            vars_["kkey2"] = edge_value(rng, 256)
            d = (kv << 512) | (vars_["kkey2"] << 256) | sv
        hv = lo + 64 * rng.randrange(1 << 20) if rng.randrange(3) else edge_value(rng, 256)
        fent = [(d, hv)] if rng.randrange(4) else []
        ient = [(hv, d)] if rng.randrange(4) else [(hv, edge_value(rng, 256))]
        return Assignment(vars=vars_,
                          funcs={fn: (fent, edge_value(rng, 256)),
                                 fn + "-1": (ient, rng.getrandbits(bits))})
    return constraints, probes, gen, {fn: 2, fn + "-1": 2}


def overflow_case():
    """Mythril's integer-overflow predicates (integer.py:143-157)."""
    from mythril_amd.smt import BVAddNoOverflow, BVMulNoOverflow, BVSubNoUnderflow, BitVec
    a, b = N.bv_var("oa", 256), N.bv_var("ob", 256)
    A, B = BitVec(a), BitVec(b)
    probes = [BVAddNoOverflow(A, B, False).raw, BVMulNoOverflow(A, B, False).raw,
              BVSubNoUnderflow(A, B, False).raw]
    constraints = [N.bool_op("not", probes[0])]

    def gen(rng):
        return Assignment(vars={"oa": edge_value(rng, 256), "ob": edge_value(rng, 256)})
    return constraints, probes, gen


def hard_division_pair(rng: random.Random):
    """(x, y) where Knuth D's two-digit quotient estimate is often two too
    big: y = a random top digit over all-ones lower digits (the shape of
    2^k - 1 boundary values), x a near multiple of y."""
    k = rng.randrange(2, 9)
    y = (1 << (32 * k - 1)) | rng.getrandbits(32 * k - 1)
    if rng.random() < 0.7:
        y |= (1 << (32 * k - 33)) - 1
    x = rng.getrandbits(256)
    if rng.random() < 0.6:
        x = (y * rng.getrandbits(32 * (8 - k) + 1) - rng.getrandbits(40)) % (1 << 256)
    if rng.random() < 0.3:                       # negative operands for the signed ops
        x = (1 << 256) - x if rng.random() < 0.5 else x
        y = (1 << 256) - y if rng.random() < 0.5 else y
    return x, y


def division_case():
    """All five division operators on hard_division_pair operands."""
    x, y = N.bv_var("dx", 256), N.bv_var("dy", 256)
    probes = [N.bv_op(op, x, y) for op in ("bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod")]
    constraints = [N.bv_cmp("bvult", probes[1], y)]

    def gen(rng):
        a, b = hard_division_pair(rng)
        return Assignment(vars={"dx": a, "dy": b})
    return constraints, probes, gen


def division_one_limb_case():
    """All five division operators with divisors that fit 32 bits in every
    lane (y & 0xffffffff and its negation): every wave takes the short
    division (asmgen._udivrem_short; the negated divisor only for the signed
    operators)."""
    x, y = N.bv_var("sx", 256), N.bv_var("sy", 256)
    d = N.bv_op("bvand", y, N.bv_num(0xFFFFFFFF, 256))
    nd = N.bv_op("bvsub", N.bv_num(0, 256), d)
    probes = [N.bv_op(op, x, dv) for dv in (d, nd)
              for op in ("bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod")]
    constraints = [N.bv_cmp("bvult", probes[1], N.bv_op("bvadd", d, N.bv_num(1, 256)))]

    def gen(rng):
        dv = rng.choice([0, 1, 3, 1 << 31, (1 << 32) - 1, rng.getrandbits(rng.choice((8, 31, 32)))])
        xv = rng.choice([0, (1 << 256) - 1, 1 << 255, rng.getrandbits(256),
                         rng.getrandbits(rng.randrange(1, 256))])
        return Assignment(vars={"sx": xv, "sy": dv | (rng.getrandbits(224) << 32)})
    return constraints, probes, gen


def const_shift_case(w: int):
    """Shifts by constants and unsigned division / remainder by powers of
    two (the forms EVM SHR/SHL/SAR/DIV/MOD by 2^k take), lowered to
    bit-field ops; constants around limb boundaries and >= w."""
    x = N.bv_var("cx%d" % w, w)
    probes = []
    for c in sorted({0, 1, 7, 31, 32, 33, w // 2, w - 1, w, w + 1, 224, 255, 256, 300}):
        k = N.bv_num(c % (1 << w), w)
        probes += [N.bv_op(op, x, k) for op in ("bvshl", "bvlshr", "bvashr")]
    for e in sorted({0, 1, 5, 32, w - 1}):
        if e < w:
            p2 = N.bv_num(1 << e, w)
            probes += [N.bv_op("bvudiv", x, p2), N.bv_op("bvurem", x, p2)]
    probes += [N.bv_op("bvudiv", x, N.bv_num(3, w)), N.bv_op("bvurem", x, N.bv_num(0, w))]
    constraints = [N.bv_cmp("bvule", probes[0], x)]

    def gen(rng):
        return Assignment(vars={x.params[0]: edge_value(rng, w)})
    return constraints, probes, gen


def named_cases():
    out = {}
    for w in WIDTHS:
        c, p, g = all_ops_case(w)
        out["ops_w%d" % w] = (c, p, g, {})
    c, p, g = bool_case()
    out["bool"] = (c, p, g, {})
    out["array"] = array_case()
    out["keccak_uf"] = keccak_uf_case()
    out["keccak_uf_768"] = keccak_uf_case(3)
    out["calldata_word"] = calldata_word_case()
    c, p, g = overflow_case()
    out["overflow"] = (c, p, g, {})
    c, p, g = division_case()
    out["division_hard"] = (c, p, g, {})
    c, p, g = division_one_limb_case()
    out["division_one_limb"] = (c, p, g, {})
    for w in (8, 160, 256):
        c, p, g = const_shift_case(w)
        out["const_shift_w%d" % w] = (c, p, g, {})
    return out
