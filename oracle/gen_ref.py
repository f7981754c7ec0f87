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
    s = (s + 0x9E3779B97F4A7C15) & M64
    z = s
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return s, z ^ (z >> 31)


CLS_MUL = 0x2545F491


def gen_class(r0: int) -> int:
    """v7: the class comes from a multiplicative remix of x = lo ^ hi of r0,
    not from bits that are emitted as value bits (v3-v6 used r0 >> 32, which
    confined bits 32-63 of the uniform / small values to their class's
    percentage band: bit 63 was never set by a random class)."""
    x = (r0 ^ (r0 >> 32)) & 0xFFFFFFFF
    return _mulhi((x * CLS_MUL) & 0xFFFFFFFF, 100)


def gen_leaf(seed: int, prog_seed: int, leaf: int, idx: int, width: int, pool,
             pct=(50, 70, 85)) -> int:
    s = (seed ^ ((prog_seed * 0xD1B54A32D192ED03) & M64) ^
         (((leaf + 1) * 0x8CB92BA72F3D8DD7) & M64) ^ idx) & M64    # v5: idx itself
    s, r0 = _sm64(s)
    # v2 range reduction: multiply-high (Lemire), no modulo
    cls = gen_class(r0)
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
