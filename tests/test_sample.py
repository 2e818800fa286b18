"""Device sampling (mhe_sample_poly, csrc/sample.hip) of the random polynomials of key
generation and encryption (util/rlwe.cpp:21 sample_poly_ternary, :72 sample_poly_normal,
:135 sample_poly_uniform).

The uniform and ternary samplers are checked bit for bit against a numpy restatement of
Philox4x32-10 (the published counter-based generator; the same counter layout as the kernel).
The normal sampler goes through device log/cos, so it is checked by its distribution: SEAL's
ClippedNormalDistribution(0, 3.2, 19.2) truncated toward zero, identical in every limb."""
import numpy as np
import pytest

import mhe
import oracle as O

M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF


def philox4x32_10(ctr, seed):
    """ctr: 4 uint64 arrays holding 32-bit words; key = (seed_lo, seed_hi)."""
    c = [x.astype(np.uint64) for x in ctr]
    k0, k1 = seed & MASK, seed >> 32
    for _ in range(10):
        p0 = c[0] * np.uint64(M0)
        p1 = c[2] * np.uint64(M1)
        h0, l0 = p0 >> np.uint64(32), p0 & np.uint64(MASK)
        h1, l1 = p1 >> np.uint64(32), p1 & np.uint64(MASK)
        c = [h1 ^ c[1] ^ np.uint64(k0), l1, h0 ^ c[3] ^ np.uint64(k1), l0]
        k0, k1 = (k0 + W0) & MASK, (k1 + W1) & MASK
    return c


def rand128(idx, tag, seed, draw=0):
    idx = idx.astype(np.uint64)
    ctr = [idx & np.uint64(MASK), (idx >> np.uint64(32)) ^ np.uint64((draw << 24) & MASK),
           np.full_like(idx, tag & MASK), np.full_like(idx, tag >> 32)]
    c = philox4x32_10(ctr, seed)
    lo = (c[1] << np.uint64(32)) | c[0]
    hi = (c[3] << np.uint64(32)) | c[2]
    return lo, hi


def test_philox_known_answer():
    # Philox4x32-10 known-answer vectors of the Random123 distribution (kat_vectors):
    # counter 0, key 0 and counter/key all-ones
    z = np.zeros(1, np.uint64)
    c = philox4x32_10([z, z, z, z], 0)
    assert [int(x[0]) for x in c] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    f = np.full(1, MASK, np.uint64)
    c = philox4x32_10([f, f, f, f], (MASK << 32) | MASK)
    assert [int(x[0]) for x in c] == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]


BITS = [51, 46, 46, 51]


@pytest.fixture(scope="module")
def eng():
    n = 1 << 12
    moduli = O.coeff_modulus_create(n, BITS)
    return mhe.Engine(12, moduli), moduli


@pytest.mark.gpu
def test_sample_uniform_bits(eng):
    e, moduli = eng
    seed, tag = 0x0123456789ABCDEF, 0xFEDCBA9876543210
    t = e.sample("uniform", len(moduli), seed, tag)
    e.synchronize()
    got = mhe.Engine.to_host(t)
    idx = np.arange(len(moduli) * e.n, dtype=np.uint64)
    lo, hi = rand128(idx, tag, seed)
    for l, q in enumerate(moduli):
        sl = slice(l * e.n, (l + 1) * e.n)
        want = [((int(h) << 64) | int(w)) % q for h, w in zip(hi[sl], lo[sl])]
        assert got[l].tolist() == want


@pytest.mark.gpu
def test_sample_ternary_bits(eng):
    e, moduli = eng
    seed, tag = 77, 5
    t = e.sample("ternary", len(moduli), seed, tag)
    e.synchronize()
    got = mhe.Engine.to_host(t)
    lo, _ = rand128(np.arange(e.n, dtype=np.uint64), tag, seed)
    v = (lo % np.uint64(3)).astype(np.int64) - 1
    for l, q in enumerate(moduli):
        want = np.where(v >= 0, v, np.int64(0)).astype(np.uint64)
        want[v < 0] = np.uint64(q - 1)
        np.testing.assert_array_equal(got[l], want)
    counts = np.bincount(v + 1, minlength=3)
    assert counts.min() > e.n / 3 * 0.9


@pytest.mark.gpu
def test_sample_normal_distribution(eng):
    e, moduli = eng
    vals = []
    for tag in range(16):
        t = e.sample("normal", len(moduli), 1234, tag)
        e.synchronize()
        got = mhe.Engine.to_host(t).astype(object)
        centered = [[int(x) if int(x) < q // 2 else int(x) - q for x in row] for row, q in zip(got, moduli)]
        for row in centered[1:]:
            assert row == centered[0]          # the same integer in every limb
        vals.extend(centered[0])
    v = np.array(vals, dtype=np.float64)
    assert np.abs(v).max() <= 19               # clipped at 6 sigma, truncated
    assert abs(v.mean()) < 0.05
    # truncation toward zero of N(0, 3.2^2) clipped at 19.2: E[trunc(z)^2] ~= 7.99
    assert 7.7 < (v * v).mean() < 8.3


@pytest.mark.gpu
def test_sample_deterministic_and_tagged(eng):
    e, moduli = eng
    a = mhe.Engine.to_host(e.sample("uniform", 2, 9, 1))
    b = mhe.Engine.to_host(e.sample("uniform", 2, 9, 1))
    c = mhe.Engine.to_host(e.sample("uniform", 2, 9, 2))
    e.synchronize()
    np.testing.assert_array_equal(a, b)
    assert (a != c).mean() > 0.99
