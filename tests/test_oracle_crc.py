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


def test_lds_tables_from_nibble_tables():
    """The identities behind stage 3's LDS tables (device_common.hpp crc_tables_lds, round 6): the
    slicing table t_k[b] (register after byte b then k zero bytes) and the zero-shift table
    z_k[i][b] = (b << 8i) * x^(8 * 16 * 2^k) (engine.cpp build_crc_consts) are GF(2)-linear in b, so
    each is nib[b & 15] ^ nib[16 + (b >> 4)]; and z_k[i] is the slicing table t_{16*2^k - 1 - i}."""
    P = 0x82F63B78

    def mulmod(a, b):
        p = 0
        for k in range(31, -1, -1):
            if (a >> k) & 1:
                p ^= b
            b = (b >> 1) ^ (P if b & 1 else 0)
        return p

    t = [[0] * 256]
    for b in range(256):
        x = b
        for _ in range(8):
            x = (x >> 1) ^ (P if x & 1 else 0)
        t[0][b] = x
    for k in range(1, 32):
        t.append([(t[k - 1][b] >> 8) ^ t[0][t[k - 1][b] & 0xFF] for b in range(256)])
    x2n = [0x40000000]
    for _ in range(8):
        x2n.append(mulmod(x2n[-1], x2n[-1]))
    z = [[[mulmod(b << (8 * i), x2n[7 + k]) for b in range(256)] for i in range(4)] for k in range(2)]
    lds = t[:8] + z[0] + z[1]  # the 16 tables in Stage3Smem order (t8, then z)
    for k in range(2):
        for i in range(4):
            assert z[k][i] == t[16 * (1 << k) - 1 - i], (k, i)
    for q, tab in enumerate(lds):
        nib = [tab[n] for n in range(16)] + [tab[n << 4] for n in range(16)]
        assert all(tab[b] == nib[b & 15] ^ nib[16 + (b >> 4)] for b in range(256)), q
