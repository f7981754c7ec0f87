"""Distribution of the device candidate generator (restated by
oracle/gen_ref.py, bit-exact with the GPU: tests/test_gpu_parity.py).

Parity tests cannot see a bias that device and oracle share; these check the
generator's own statistics.  Generator v3-v6 drew the class from r0 >> 32,
which also supplied value bits 32-63, so bit 63 was never set by the random
classes; v7 draws it from a remix of lo ^ hi.
"""

import pytest

from oracle import gen_ref

N = 20000
M64 = (1 << 64) - 1


def _draws(pct=(50, 70, 85)):
    pool = [0x1234, 1 << 200]
    out = {"uniform": [], "small": [], "boundary": 0, "pool": 0}
    for i in range(N):
        seed, leaf, idx = 0xC0FFEE, i % 7, 1000 + i
        s = (seed ^ ((3 * 0xD1B54A32D192ED03) & M64) ^
             (((leaf + 1) * 0x8CB92BA72F3D8DD7) & M64) ^ idx) & M64
        _, r0 = gen_ref._sm64(s)
        cls = gen_ref.gen_class(r0)
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
