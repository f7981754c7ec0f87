"""ORACLE — test infrastructure only.

Host restatement of the device candidate generator (``_gen_leaf`` in
``mythril_amd/asmgen.py``; contract in ``include/mythgpu.h``
``mg_leafgen``), so tests can rebuild the exact assignment a GPU lane
evaluated and check the lane against ``oracle/smtlib_ref.py``.
"""

M64 = (1 << 64) - 1


def _mulhi(a, b):
    return (a * b) >> 32


def _sm64(s):
    """v9 mixer: s += GOLD; u = s ^ (s >> 32); z = u * MIX1; r0 = z ^ (z >> 32)
    (all mod 2^64; v5-v8 ran SplitMix64's finaliser)."""
    s = (s + 0x9E3779B97F4A7C15) & M64
    u = s ^ (s >> 32)
    z = (u * 0xBF58476D1CE4E5B9) & M64
    return s, z ^ (z >> 32)


CLS_MUL = 0x2545F491


def gen_class(seed: int, prog_seed: int, leaf: int, idx: int) -> int:
    """v8: the class is drawn once per leaf per GROUP of 64 consecutive
    candidate indices (idx >> 6: the candidates of one wave when a launch
    starts at a multiple of 64, which every search / bench launch does), so
    a wave evaluates one class's code instead of all four under exec:
      ss  = seed ^ salt
      y   = ((lo32(idx >> 6) ^ lo32(ss)) * CLS_MUL) ^ hi32(ss)   (mod 2^32)
      cls = mulhi(y, 100)
    v7 drew it per lane from a remix of r0 (and v3-v6 from r0 >> 32, which
    confined value bits 32-63 to the class's band); the value bits still
    come from r0 alone."""
    ss = (seed ^ _salt(prog_seed, leaf)) & M64
    w = (idx >> 6) & 0xFFFFFFFF
    y = ((((w ^ ss) & 0xFFFFFFFF) * CLS_MUL) & 0xFFFFFFFF) ^ (ss >> 32)
    return _mulhi(y, 100)


def _salt(prog_seed: int, leaf: int) -> int:
    return ((prog_seed * 0xD1B54A32D192ED03) & M64) ^ (((leaf + 1) * 0x8CB92BA72F3D8DD7) & M64)


def gen_leaf(seed: int, prog_seed: int, leaf: int, idx: int, width: int, pool,
             pct=(50, 70, 85)) -> int:
    s = (seed ^ _salt(prog_seed, leaf) ^ idx) & M64    # v5: idx itself
    s, r0 = _sm64(s)
    # v2 range reduction: multiply-high (Lemire), no modulo; v8: the class
    # per 64-candidate group
    cls = gen_class(seed, prog_seed, leaf, idx)
    lo = r0 & 0xFFFFFFFF
    mask = (1 << width) - 1
    if pct[0] <= cls < pct[1]:
        v = r0                                # v3: the class word itself
    elif pct[1] <= cls < pct[2]:
        kind = _mulhi(lo, 6)
        k = _mulhi((lo * 0x9E3779B1) & 0xFFFFFFFF, width)
        v = {0: 0, 1: 1, 2: 1 << (width - 1), 3: (1 << 256) - 1,
             4: (1 << k) + 1, 5: (1 << k) - 1}[kind]
    elif cls >= pct[2] and len(pool) > 0:
        e = _mulhi(lo, len(pool))
        delta = _mulhi((lo * 0x85EBCA6B) & 0xFFFFFFFF, 3)
        v = (pool[e] + delta - 1) % (1 << 256)
    else:
        v = r0                                # v6: limb pair k = x * C_k + r0
        x = (r0 ^ (r0 >> 32)) & 0xFFFFFFFF
        for k, c in enumerate((0x85EBCA6B, 0xC2B2AE35, 0x27D4EB2F)):
            v |= ((x * c + r0) & M64) << (64 * (k + 1))
    return v & mask
