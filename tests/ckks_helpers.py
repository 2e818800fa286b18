"""Test-side CKKS helpers: key generation, symmetric encryption, decryption and a
canonical-embedding encoder/decoder, composed from the oracle's per-limb primitives.

These make decryptable inputs for the end-to-end sanity checks (SURVEY.md §8(d) input
kind (ii)).  They follow the reference's algorithms structurally --
keygenerator.cpp:384-414 (one kswitch key per data limb, P mod q_J times the new key added
to limb J of c0), rlwe.cpp:40-70 (sparse ternary secret, clipped rounded Gaussian error),
encryptor/decryptor semantics -- but use numpy's seeded PRNG instead of Blake2xb, so the
keys are not the bits SEAL would draw: parity of *ciphertext operations* never depends on
that (every op is a deterministic function of its inputs), only decryptability does.
"""
import numpy as np

import oracle as O

NOISE_STD = 3.2          # util/globals.h:36 (seal_he_std_parms_error_std_dev)
NOISE_MAX = 3.2 * 6      # util/globals.h:38-40


class Keys:
    pass


def _residues(coeffs, moduli):
    """int64 coefficient vector -> [len(moduli)][n] canonical residues."""
    c = np.asarray(coeffs, dtype=np.int64)
    out = np.empty((len(moduli), c.size), np.uint64)
    for i, q in enumerate(moduli):
        out[i] = np.mod(c, np.int64(q)).astype(np.uint64)
    return out


def uniform(rng, moduli, n):
    out = np.empty((len(moduli), n), np.uint64)
    for i, q in enumerate(moduli):
        out[i] = rng.integers(0, q, size=n, dtype=np.uint64)
    return out


def gaussian(rng, n):
    e = np.rint(rng.normal(0.0, NOISE_STD, size=n))
    return np.clip(e, -NOISE_MAX, NOISE_MAX).astype(np.int64)


def sparse_ternary(rng, n, hw):
    s = np.zeros(n, np.int64)
    pos = rng.choice(n, size=hw, replace=False)
    s[pos] = rng.choice(np.array([-1, 1], np.int64), size=hw)
    return s


def keygen(ctx, seed=1, hw=192):
    """Secret key (NTT form over the key chain), relin key for s^2."""
    rng = np.random.default_rng(seed)
    k = Keys()
    k.ctx = ctx
    k.rng = rng
    k.s_coeff = sparse_ternary(rng, ctx.n, hw)
    k.s = ctx.ntt(_residues(k.s_coeff, ctx.moduli))          # [K][n]
    k.s2 = ctx.dyadic(k.s, k.s)
    k.relin = kswitch_key(ctx, k, k.s2)
    return k


def kswitch_key(ctx, keys, new_key_ntt):
    """KeyGenerator::generate_one_kswitch_key (keygenerator.cpp:384-414):
    key[J] = (-(a s) + e + [J] (P mod q_J) s', a), shape [K-1][2][K][n]."""
    K, n = ctx.k, ctx.n
    P = ctx.moduli[-1]
    key = np.empty((K - 1, 2, K, n), np.uint64)
    for J in range(K - 1):
        a = uniform(keys.rng, ctx.moduli, n)
        e = ctx.ntt(_residues(gaussian(keys.rng, n), ctx.moduli))
        c0 = ctx.add(ctx.negate(ctx.dyadic(a, keys.s)), e)
        fac = np.zeros((K, n), np.uint64)
        fac[J] = P % ctx.moduli[J]
        c0 = ctx.add(c0, ctx.dyadic(fac, new_key_ntt))
        key[J, 0] = c0
        key[J, 1] = a
    return key


def galois_key(ctx, keys, elt):
    """Galois key for element elt: kswitch key of s(X^elt) (keygenerator.cpp create_galois_keys)."""
    perm = O.apply_galois_ntt(keys.s, ctx.log_n, elt)
    return kswitch_key(ctx, keys, perm)


def encrypt(ctx, keys, pt, L):
    """Symmetric encryption of an NTT-form plaintext pt [L][n] at L data limbs."""
    mods = ctx.moduli[:L]
    a = uniform(keys.rng, mods, ctx.n)
    e = ctx.ntt(_residues(gaussian(keys.rng, ctx.n), mods))
    s = keys.s[:L]
    c0 = ctx.add(ctx.add(ctx.negate(ctx.dyadic(a, s)), e), pt)
    return np.stack([c0, a])


def decrypt(ctx, keys, ct):
    """Decryptor::decrypt for size-2/3 CKKS ct: c0 + c1 s (+ c2 s^2), NTT form [L][n]."""
    L = ct.shape[1]
    m = ctx.add(ct[0], ctx.dyadic(ct[1], keys.s[:L]))
    if ct.shape[0] == 3:
        m = ctx.add(m, ctx.dyadic(ct[2], keys.s2[:L]))
    return m


# ----------------------------------------------------------------------- encode / decode
def _slot_index(n):
    """Slot i <-> evaluation at zeta^(5^i mod 2n) (ckks.cpp:34-49)."""
    m = 2 * n
    k = np.empty(n // 2, np.int64)
    pos = 1
    for i in range(n // 2):
        k[i] = pos
        pos = (pos * 5) % m
    return (k - 1) // 2, (m - k - 1) // 2


def encode(ctx, values, scale, L):
    """Real/complex slots -> NTT-form plaintext [L][n] (canonical embedding; not SEAL's
    exact FFT rounding -- only used to make decryptable test inputs)."""
    n = ctx.n
    t1, t2 = _slot_index(n)
    v = np.zeros(n, np.complex128)
    z = np.zeros(n // 2, np.complex128)
    z[: len(values)] = values
    v[t1] = z
    v[t2] = np.conj(z)
    j = np.arange(n)
    zeta = np.exp(1j * np.pi * j / n)
    coeff = (np.fft.fft(v) / n) * np.conj(zeta)
    c = np.rint(coeff.real * scale).astype(np.int64)
    return ctx.ntt(_residues(c, ctx.moduli[:L]))


def decode(ctx, pt, scale):
    """NTT-form plaintext -> slots, using limb 0 only (values must be < q_0/2)."""
    n = ctx.n
    q0 = ctx.moduli[0]
    c = ctx.ntt(pt[:1], O.NTT_INV)[0].astype(np.int64)
    c = np.where(c > q0 // 2, c - np.int64(q0), c).astype(np.float64) / scale
    j = np.arange(n)
    zeta = np.exp(1j * np.pi * j / n)
    ev = n * np.fft.ifft(c * zeta)
    t1, _ = _slot_index(n)
    return ev[t1]
