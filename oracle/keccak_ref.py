"""ORACLE — test infrastructure only.

Keccak-256 as used by the reference for concrete hashes:
``mythril/laser/ethereum/keccak_function_manager.py:43-57`` calls
``ethereum.utils.sha3`` (third-party ``ethereum>=2.3.2``, ``requirements.txt:7``;
not vendored, not installed here), which is Keccak-256 with the original
``0x01`` multi-rate padding (not FIPS-202 SHA3's ``0x06``).

Restated from the published Keccak reference (Keccak-f[1600], 24 rounds,
rate 1088 bits, capacity 512).  Pinned by (a) ``hashlib.sha3_256`` — same
permutation, 0x06 padding — through :func:`sha3_256_fips`, and (b) the
Keccak-256 answers in ``vmSha3Test`` (``tests/golden/keccak_kat.json``) and
``keccak_function_manager.py:80`` (the empty-string hash).
"""

_RC = [
    0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
    0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
    0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
    0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
    0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
    0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008,
]

# rotation offsets r[x][y]
_ROT = [
    [0, 36, 3, 41, 18],
    [1, 44, 10, 45, 2],
    [62, 6, 43, 15, 61],
    [28, 55, 25, 21, 56],
    [27, 20, 39, 8, 14],
]

M64 = (1 << 64) - 1


def _rol(v, n):
    n %= 64
    return ((v << n) | (v >> (64 - n))) & M64 if n else v


def keccak_f1600(A):
    """A: list of 25 lanes, index x + 5*y."""
    for rnd in range(24):
        C = [A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20] for x in range(5)]
        D = [C[(x - 1) % 5] ^ _rol(C[(x + 1) % 5], 1) for x in range(5)]
        A = [A[i] ^ D[i % 5] for i in range(25)]
        B = [0] * 25
        for x in range(5):
            for y in range(5):
                B[y + 5 * ((2 * x + 3 * y) % 5)] = _rol(A[x + 5 * y], _ROT[x][y])
        A = [B[i] ^ ((~B[(i % 5 + 1) % 5 + 5 * (i // 5)]) & B[(i % 5 + 2) % 5 + 5 * (i // 5)])
             for i in range(25)]
        A[0] ^= _RC[rnd]
    return A


def _sponge(msg: bytes, pad_byte: int, rate: int = 136, out_len: int = 32) -> bytes:
    data = bytearray(msg)
    data.append(pad_byte)
    while len(data) % rate:
        data.append(0)
    data[-1] |= 0x80
    A = [0] * 25
    for off in range(0, len(data), rate):
        block = data[off:off + rate]
        for i in range(rate // 8):
            A[i] ^= int.from_bytes(block[8 * i:8 * i + 8], "little")
        A = keccak_f1600(A)
    out = b"".join(A[i].to_bytes(8, "little") for i in range(rate // 8))
    return out[:out_len]


def keccak256(msg: bytes) -> bytes:
    return _sponge(msg, 0x01)


def sha3_256_fips(msg: bytes) -> bytes:
    return _sponge(msg, 0x06)
