"""The oracle's CRC32C against RFC 3720 §B.4 known answers, and table/SSE4.2 vs bitwise."""
import numpy as np
import pytest

from kat import vectors


@pytest.mark.parametrize("name,data,expected", vectors())
def test_rfc3720_vectors(oracle_mod, name, data, expected):
    assert oracle_mod.crc32c(data, bitwise=True) == expected
    assert oracle_mod.crc32c(data) == expected


def test_fast_matches_bitwise(oracle_mod):
    g = np.random.default_rng(1)
    for n in list(range(0, 70)) + [100, 255, 1000, 4099, 16384]:
        d = g.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert oracle_mod.crc32c(d) == oracle_mod.crc32c(d, bitwise=True), n


def test_crc_combine_identity(oracle_mod):
    # crc(A||B) = shift(crc(A), |B|) ^ crc(B): the GF(2) identity the wave-parallel kernel uses
    P = 0x82F63B78

    def mulmod(a, b):
        p = 0
        for k in range(31, -1, -1):
            if (a >> k) & 1:
                p ^= b
            b = (b >> 1) ^ (P if b & 1 else 0)
        return p

    x2n = [0x40000000]
    for _ in range(40):
        x2n.append(mulmod(x2n[-1], x2n[-1]))

    def shift(c, n):
        j = 0
        while n:
            if n & 1:
                c = mulmod(x2n[j + 3], c)
            n >>= 1
            j += 1
        return c

    g = np.random.default_rng(2)
    for la, lb in [(0, 5), (5, 0), (1, 1), (100, 37), (4096, 3), (77, 16384)]:
        a = g.integers(0, 256, la, dtype=np.uint8).tobytes()
        b = g.integers(0, 256, lb, dtype=np.uint8).tobytes()
        got = shift(oracle_mod.crc32c(a), lb) ^ oracle_mod.crc32c(b)
        assert got == oracle_mod.crc32c(a + b)
