"""The oracle's CKKS encoder restatement (ckks.h:457-640) is a correct CKKS encoder: it decodes
back to the input (canonical-embedding decode, tests/ckks_helpers.decode), handles complex
input, all three coefficient-width paths (<=64, <=128, multi-word), and SEAL's range checks."""
import numpy as np
import pytest

import ckks_helpers as H
import oracle as O


@pytest.fixture(scope="module")
def ctx():
    log_n = 12
    return O.Context(log_n, O.coeff_modulus_create(1 << log_n, [60, 40, 40, 40, 60]))


def test_encode_real_roundtrip(ctx):
    x = np.random.default_rng(0).uniform(-1, 1, ctx.n // 2)
    pt = ctx.encode(x, 2.0 ** 30, 4)
    assert np.abs(H.decode(ctx, pt, 2.0 ** 30) - x).max() < 1e-6


def test_encode_complex_roundtrip(ctx):
    rng = np.random.default_rng(1)
    z = rng.uniform(-1, 1, ctx.n // 2) + 1j * rng.uniform(-1, 1, ctx.n // 2)
    pt = ctx.encode(z, 2.0 ** 30, 4)
    assert np.abs(H.decode(ctx, pt, 2.0 ** 30) - z).max() < 1e-6


def test_encode_matches_helper_encoder(ctx):
    """Same rounded coefficients as an independent canonical-embedding encoder up to +-1."""
    x = np.random.default_rng(2).uniform(-1, 1, ctx.n // 2)
    a = ctx.ntt(ctx.encode(x, 2.0 ** 30, 1), O.NTT_INV)[0].astype(np.int64)
    b = ctx.ntt(H.encode(ctx, x, 2.0 ** 30, 1), O.NTT_INV)[0].astype(np.int64)
    q = ctx.moduli[0]
    d = (a - b) % q
    assert np.all((d <= 1) | (d >= q - 1))


def _crt(c, moduli, idx):
    """CRT-compose coefficient idx of a coefficient-form RNS polynomial, centred."""
    Q = 1
    for q in moduli:
        Q *= q
    x = 0
    for l, q in enumerate(moduli):
        Qi = Q // q
        x += int(c[l, idx]) * Qi * pow(Qi, -1, q)
    x %= Q
    return x - Q if x > Q // 2 else x


def test_encode_wide_paths(ctx):
    """scale 2^70 forces the 128-bit path, 2^140 the multi-word path (ckks.h:560-628); the
    CRT-composed integer coefficients match an independent float encoder to ~1e-12."""
    x = np.random.default_rng(3).uniform(-1, 1, ctx.n // 2)
    ref = ctx.ntt(H.encode(ctx, x, 1.0 * 2 ** 20, 1), O.NTT_INV)[0].astype(np.int64)  # shape of coefficients
    for scale in (2.0 ** 70, 2.0 ** 140):
        c = ctx.ntt(ctx.encode(x, scale, 5), O.NTT_INV)
        for idx in range(0, ctx.n, 257):
            got = _crt(c, ctx.moduli[:5], idx)
            want = int(ref[idx] if ref[idx] < ctx.moduli[0] // 2 else ref[idx] - ctx.moduli[0]) * (scale / 2 ** 20)
            assert abs(got - want) <= 1e-5 * scale


def test_encode_scale_out_of_bounds(ctx):
    with pytest.raises(ValueError, match="scale out of bounds"):
        ctx.encode([1.0], 2.0 ** 300, 4)


def test_encode_scalar(ctx):
    r = ctx.encode_scalar(-0.75, 2.0 ** 40, 3)
    for q, v in zip(ctx.moduli, r):
        assert (v - (q - round(0.75 * 2 ** 40))) % q == 0
    r = ctx.encode_scalar(3.0, 2.0 ** 100, 4)  # 128-bit path
    for q, v in zip(ctx.moduli, r):
        assert v == (3 * 2 ** 100) % q


# ----------------------------------------------------------------------------- decode
def test_decode_roundtrip_real_and_complex(ctx):
    rng = np.random.default_rng(11)
    x = rng.uniform(-1, 1, ctx.n // 2)
    assert np.abs(ctx.decode(ctx.encode(x, 2.0 ** 30, 4), 2.0 ** 30).real - x).max() < 1e-6
    z = rng.uniform(-1, 1, ctx.n // 2) + 1j * rng.uniform(-1, 1, ctx.n // 2)
    assert np.abs(ctx.decode(ctx.encode(z, 2.0 ** 30, 3), 2.0 ** 30) - z).max() < 1e-6


def test_decode_matches_bigint_crt(ctx):
    """CRT compose + centered lift agrees with an independent Python-int reconstruction on a
    plaintext whose coefficients span the whole modulus (multi-limb values of both signs)."""
    L = 3
    rng = np.random.default_rng(12)
    x = rng.uniform(-1, 1, ctx.n // 2) * 2.0 ** 40
    pt = ctx.encode(x, 2.0 ** 60, L)  # |coeff| ~ 2^100: needs all three limbs
    got = ctx.decode(pt, 2.0 ** 60)
    c = ctx.ntt(pt, O.NTT_INV)
    Q = 1
    for q in ctx.moduli[:L]:
        Q *= q
    vals = []
    for i in range(ctx.n):
        v = 0
        for j, q in enumerate(ctx.moduli[:L]):
            Mj = Q // q
            v += int(c[j, i]) * pow(Mj, -1, q) * Mj
        v %= Q
        vals.append(float(v - Q if v > Q // 2 else v) / 2.0 ** 60)
    coeff = np.array(vals)
    n = ctx.n
    zeta = np.exp(1j * np.pi * np.arange(n) / n)
    ev = n * np.fft.ifft(coeff * zeta)
    t1, _ = H._slot_index(n)
    ref = ev[t1]
    assert np.abs(got - ref).max() < 1e-6 * np.abs(ref).max()
    assert np.abs(got.real - x).max() < 1e-6 * 2.0 ** 40


def test_decode_single_limb(ctx):
    x = np.random.default_rng(13).uniform(-1, 1, ctx.n // 2)
    assert np.abs(ctx.decode(ctx.encode(x, 2.0 ** 30, 1), 2.0 ** 30).real - x).max() < 1e-6


def test_decode_sparse_slots(ctx):
    """Modified SEAL sparse decode (ckks.h:704-713): a vector with period `sparse` in the slots
    lives on coefficients i = 0 mod (slots/sparse); decode returns the first `sparse` slots."""
    sparse = 64
    rng = np.random.default_rng(14)
    base = rng.uniform(-1, 1, sparse)
    x = np.tile(base, ctx.n // 2 // sparse)
    out = ctx.decode(ctx.encode(x, 2.0 ** 30, 2), 2.0 ** 30, sparse_slots=sparse)
    assert out.shape == (sparse,)
    assert np.abs(out.real - base).max() < 1e-6


def test_decode_scale_bounds(ctx):
    pt = ctx.encode([0.5], 2.0 ** 30, 1)
    with pytest.raises(ValueError, match="scale out of bounds"):
        ctx.decode(pt, 2.0 ** 70)
