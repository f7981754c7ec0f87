"""Distribution of the device candidate generator (restated by
oracle/gen_ref.py, bit-exact with the GPU: tests/test_gpu_parity.py).

Parity tests cannot see a bias that device and oracle share; these check the
generator's own statistics.  Generator v3-v6 drew the class from r0 >> 32,
which also supplied value bits 32-63, so bit 63 was never set by the random
classes; v7 drew it per lane from a remix of lo ^ hi; v8
draws it per leaf per group of 64 consecutive indices (one class per wave),
so the draws below take one index from each group.
"""

import pytest

from oracle import gen_ref

N = 20000
M64 = (1 << 64) - 1


def _draws(pct=(50, 70, 85)):
    pool = [0x1234, 1 << 200]
    out = {"uniform": [], "small": [], "boundary": 0, "pool": 0}
    for i in range(N):
        seed, leaf, idx = 0xC0FFEE, i % 7, 1000 + 64 * i + i % 64
        cls = gen_ref.gen_class(seed, 3, leaf, idx)
        v = gen_ref.gen_leaf(seed, 3, leaf, idx, 256, pool, pct)
        if cls < pct[0]:
            out["uniform"].append(v)
        elif cls < pct[1]:
            out["small"].append(v)
        elif cls < pct[2]:
            out["boundary"] += 1
        else:
            out["pool"] += 1
    return out


@pytest.fixture(scope="module")
def draws():
    return _draws()


def test_class_frequencies(draws):
    n_u, n_s = len(draws["uniform"]), len(draws["small"])
    for got, want in ((n_u, 0.50), (n_s, 0.20), (draws["boundary"], 0.15), (draws["pool"], 0.15)):
        assert abs(got / N - want) < 0.015, (got, want)


@pytest.mark.parametrize("bit", [31, 32, 56, 60, 62, 63, 64, 127, 191, 255])
def test_uniform_value_bits_are_balanced(draws, bit):
    vals = draws["uniform"]
    frac = sum((v >> bit) & 1 for v in vals) / len(vals)
    assert abs(frac - 0.5) < 0.025, (bit, frac)


@pytest.mark.parametrize("bit", [31, 48, 62, 63])
def test_small_value_bits_are_balanced(draws, bit):
    vals = draws["small"]
    assert all(v < (1 << 64) for v in vals)
    frac = sum((v >> bit) & 1 for v in vals) / len(vals)
    assert abs(frac - 0.5) < 0.035, (bit, frac)


def test_top_byte_of_hi32_covers_the_range(draws):
    # v6: the uniform class confined hi32 to [0, 0.5 * 2^32) (cls < 50)
    tops = {(v >> 56) & 0xFF for v in draws["uniform"]}
    assert len(tops) == 256
    big = sum(1 for v in draws["uniform"] if (v & M64) >= (1 << 63) + (1 << 62))
    assert abs(big / len(draws["uniform"]) - 0.25) < 0.025


def test_class_is_constant_over_a_group_of_64():
    seed, pool = 0xBEEF, [5, 1 << 100]
    for leaf in range(4):
        for g in range(50):
            base = 64 * (g + 1000)
            cls = {gen_ref.gen_class(seed, 9, leaf, base + j) for j in range(64)}
            assert len(cls) == 1
            vals = {gen_ref.gen_leaf(seed, 9, leaf, base + j, 256, pool) for j in range(64)}
            # the value bits still vary per candidate (boundary: 6 kinds x k)
            assert len(vals) > 3


def test_leaves_draw_independent_classes():
    # two leaves of one program must not share the group's class sequence
    seed = 0x5EED
    a = [gen_ref.gen_class(seed, 1, 0, 64 * g) for g in range(4000)]
    b = [gen_ref.gen_class(seed, 1, 1, 64 * g) for g in range(4000)]
    same = sum(x // 50 == y // 50 for x, y in zip(a, b)) / len(a)
    assert abs(same - 0.5) < 0.04
