"""GPU parity: the HIP engine (through the C ABI of include/mhe.h) against the CPU oracle,
bit for bit, on seeded inputs.  Sizes: N=2^12 (fast, every op and edge case), and the full
N=2^16 chains of the reference -- the 45-prime C2 chain, the ResNet
chain (cnn/infer_seal.cpp:288-316) and the GPT-2 chain with its 60-bit special prime
(gpt2/util.h:22-27).  Names follow the reference GoogleTest / evaluator entry points."""
import numpy as np
import pytest

import ckks_helpers as H
import mhe
import oracle as O

pytestmark = pytest.mark.gpu

C2_BITS = [51] + [46] * 30 + [51] * 13 + [51]       # 44 data limbs + special
RESNET_BITS = [51] + [46] * 16 + [51] * 14 + [51]   # 31 data limbs + special
GPT2_BITS = [49] + [46] * 21 + [49] * 14 + [60]     # 36 data limbs + 60-bit special
SMALL_BITS = [51] + [46] * 4 + [51] * 2 + [51]      # 7 data limbs + special


class Chain:
    def __init__(self, log_n, bits, seed=0):
        self.log_n, self.n = log_n, 1 << log_n
        self.moduli = O.coeff_modulus_create(self.n, bits)
        self.K = len(self.moduli)
        self.oc = O.Context(log_n, self.moduli)
        self.eng = mhe.Engine(log_n, self.moduli)
        self.rng = np.random.default_rng(seed)

    def rand(self, *shape, limbs=None):
        """Uniform residues, shape [..., limbs, n] with limb l mod q_l."""
        L = shape[-2]
        out = np.empty(shape, np.uint64)
        for l in range(L):
            out[..., l, :] = self.rng.integers(0, self.moduli[l], size=shape[:-2] + (self.n,), dtype=np.uint64)
        return out

    def rand_key(self, digits=None):
        """Random key-switching key [digits][2][K][n] (uniform residues per key-level prime)."""
        digits = self.K - 1 if digits is None else digits
        key = np.empty((digits, 2, self.K, self.n), np.uint64)
        for l, q in enumerate(self.moduli):
            key[:, :, l, :] = self.rng.integers(0, q, size=(digits, 2, self.n), dtype=np.uint64)
        return key

    def up(self, a):
        return self.eng.to_device(a)

    def down(self, t):
        self.eng.synchronize()
        return mhe.Engine.to_host(t)


@pytest.fixture(scope="module")
def small():
    return Chain(12, SMALL_BITS, seed=1)


@pytest.fixture(scope="module")
def c2():
    return Chain(16, C2_BITS, seed=2)


# ----------------------------------------------------------------------------- NTT
@pytest.mark.parametrize("lazy", [False, True])
def test_ntt_negacyclic_harvey(small, lazy):
    ch = small
    x = ch.rand(3, ch.K - 1, ch.n)
    got = ch.down(ch.eng.ntt_forward(ch.up(x), lazy=lazy))
    want = ch.oc.ntt(x, O.NTT_FWD)
    if lazy:
        assert (got < 4 * np.array(ch.moduli[:-1], np.uint64)[None, :, None]).all()
        got = got % np.array(ch.moduli[:-1], np.uint64)[None, :, None]
    assert np.array_equal(got, want)


@pytest.mark.parametrize("lazy", [False, True])
def test_inverse_ntt_negacyclic_harvey(small, lazy):
    ch = small
    x = ch.rand(2, ch.K, ch.n)
    got = ch.down(ch.eng.ntt_inverse(ch.up(x), lazy=lazy))
    want = ch.oc.ntt(x, O.NTT_INV)
    if lazy:
        got = got % np.array(ch.moduli, np.uint64)[None, :, None]
    assert np.array_equal(got, want)


@pytest.mark.parametrize("log_n", [12, 13, 14, 15, 16])
def test_ntt_all_sizes(log_n):
    """Every supported ring degree (column/row pass split differs for odd log n)."""
    moduli = O.coeff_modulus_create(1 << log_n, [50, 40, 60])
    oc = O.Context(log_n, moduli)
    eng = mhe.Engine(log_n, moduli)
    rng = np.random.default_rng(log_n)
    x = np.stack([rng.integers(0, q, size=1 << log_n, dtype=np.uint64) for q in moduli])
    t = eng.to_device(x)
    eng.ntt_forward(t)
    eng.synchronize()
    got = mhe.Engine.to_host(t)
    assert np.array_equal(got, oc.ntt(x, O.NTT_FWD))
    eng.ntt_inverse(t)
    eng.synchronize()
    assert np.array_equal(mhe.Engine.to_host(t), x)


def test_ntt_kat_vectors():
    """The reference KAT modulus 0xffffffffffc0001 at N=2^12: GPU == oracle, round trip exact."""
    q = 0xFFFFFFFFFFC0001
    # q-1 = 2^18 * ... so q is NTT-friendly for 2n <= 2^18
    eng = mhe.Engine(12, [q, O.get_primes(1 << 12, 50, 1)[0]])
    x = np.random.default_rng(7).integers(0, q, size=(1, 1 << 12), dtype=np.uint64)
    t = eng.to_device(x)
    eng.ntt_forward(t)
    eng.synchronize()
    assert np.array_equal(mhe.Engine.to_host(t), O.ntt(x, 12, q).reshape(1, -1))


# ---------------------------------------------------------------- coefficient-wise
def test_add_sub_negate(small):
    ch = small
    a, b = ch.rand(2, ch.K - 1, ch.n), ch.rand(2, ch.K - 1, ch.n)
    ta, tb = ch.up(a), ch.up(b)
    assert np.array_equal(ch.down(ch.eng.add(ta, tb)), ch.oc.add(a, b))
    assert np.array_equal(ch.down(ch.eng.sub(ta, tb)), ch.oc.sub(a, b))
    assert np.array_equal(ch.down(ch.eng.negate(ta)), ch.oc.negate(a))
    # in place (out aliases a)
    ch.eng.add(ta, tb, out=ta)
    assert np.array_equal(ch.down(ta), ch.oc.add(a, b))


def test_multiply_plain_ntt(small):
    ch = small
    L = ch.K - 1
    ct, pt = ch.rand(2, L, ch.n), ch.rand(L, ch.n)
    got = ch.down(ch.eng.multiply_plain(ch.up(ct), ch.up(pt)))
    assert np.array_equal(got, ch.oc.multiply_plain(ct, pt))


@pytest.mark.parametrize("terms", [1, 9, 17])
def test_multiply_plain_sum(small, terms):
    """mhe_multiply_plain_sum == multiply_plain of the first term + add of each later product
    (the conv taps / BSGS inner sums), also past the 16 terms of one launch and accumulating."""
    ch = small
    L = ch.K - 1
    cts = [ch.rand(2, L, ch.n) for _ in range(terms)]
    pts = [ch.rand(L, ch.n) for _ in range(terms)]
    want = ch.oc.multiply_plain(cts[0], pts[0])
    for c, p in zip(cts[1:], pts[1:]):
        want = ch.oc.add(want, ch.oc.multiply_plain(c, p))
    dc, dp = [ch.up(c) for c in cts], [ch.up(p) for p in pts]
    got = ch.down(ch.eng.multiply_plain_sum(dc, dp))
    assert np.array_equal(got, want)
    acc = ch.rand(2, L, ch.n)
    got2 = ch.down(ch.eng.multiply_plain_sum(dc, dp, out=ch.up(acc), accumulate=True))
    assert np.array_equal(got2, ch.oc.add(acc, want))


@pytest.mark.parametrize("env", [{}, {"MHE_FP": "0"}], ids=["fp64", "integer"])
def test_elementwise_products_both_paths(env):
    """The elementwise products -- multiply_plain, the multi-term product sum (past 16 terms,
    accumulating), ckks_multiply / ckks_square -- in the FP64 path (primes below 2^51, round 6) and
    the integer path (MHE_FP=0), on residues that include 0 and q - 1 in every limb: bit-identical to
    the oracle both ways."""
    ch = _variant_chain(env, 91)
    L = ch.K - 1
    qs = np.array(ch.moduli[:L], np.uint64)

    a, b = ch.rand(2, L, ch.n), ch.rand(2, L, ch.n)
    for x in (a, b):
        x[:, :, 0] = 0
        x[:, :, 1] = (qs - np.uint64(1))[None, :]
    pt = ch.rand(L, ch.n)
    pt[:, 1] = qs - np.uint64(1)
    assert np.array_equal(ch.down(ch.eng.multiply_plain(ch.up(a), ch.up(pt))), ch.oc.multiply_plain(a, pt))
    assert np.array_equal(ch.down(ch.eng.multiply(ch.up(a), ch.up(b))), ch.oc.multiply(a, b))
    assert np.array_equal(ch.down(ch.eng.square(ch.up(a))), ch.oc.square(a))
    cts = [a if k % 2 else b for k in range(18)]
    pts = [pt] * 18
    want = ch.oc.multiply_plain(cts[0], pts[0])
    for c, p in zip(cts[1:], pts[1:]):
        want = ch.oc.add(want, ch.oc.multiply_plain(c, p))
    acc = b.copy()
    got = ch.down(ch.eng.multiply_plain_sum([ch.up(c) for c in cts], [ch.up(p) for p in pts], out=ch.up(acc),
                                            accumulate=True))
    assert np.array_equal(got, ch.oc.add(acc, want))


def test_multiply_add_scalar(small):
    ch = small
    L = ch.K - 1
    a = ch.rand(2, L, ch.n)
    s = [int(ch.rng.integers(0, q)) for q in ch.moduli[:L]]
    got = ch.down(ch.eng.multiply_scalar(ch.up(a), s))
    want = np.stack([np.stack([(a[p, l].astype(object) * s[l] % ch.moduli[l]).astype(np.uint64) for l in range(L)])
                     for p in range(2)])
    assert np.array_equal(got, want)
    got = ch.down(ch.eng.add_scalar(ch.up(a), s))
    want = np.stack([np.stack([((a[p, l].astype(object) + s[l]) % ch.moduli[l]).astype(np.uint64) for l in range(L)])
                     for p in range(2)])
    assert np.array_equal(got, want)


# ----------------------------------------------------------------- ciphertext ops
@pytest.mark.parametrize("L", [1, 4, 7])
def test_ckks_multiply(small, L):
    ch = small
    a, b = ch.rand(2, L, ch.n), ch.rand(2, L, ch.n)
    got = ch.down(ch.eng.multiply(ch.up(a), ch.up(b)))
    assert np.array_equal(got, ch.oc.multiply(a, b))


def test_ckks_square(small):
    ch = small
    a = ch.rand(2, 5, ch.n)
    got = ch.down(ch.eng.square(ch.up(a)))
    assert np.array_equal(got, ch.oc.square(a))


@pytest.mark.parametrize("L", [2, 3, 7])
@pytest.mark.parametrize("size", [1, 2, 3])
def test_rescale_to_next(small, L, size):
    ch = small
    ct = ch.rand(size, L, ch.n)
    got = ch.down(ch.eng.rescale_to_next(ch.up(ct)))
    assert np.array_equal(got, ch.oc.rescale(ct))


@pytest.mark.parametrize("L", [1, 2, 5, 7])
def test_switch_key_inplace(small, L):
    ch = small
    key = ch.rand_key()
    ct, target = ch.rand(2, L, ch.n), ch.rand(L, ch.n)
    got = ch.down(ch.eng.switch_key(ch.up(ct), ch.up(target), ch.up(key)))
    assert np.array_equal(got, ch.oc.switch_key(ct, target, key))


def test_switch_key_truncated_key(small):
    """A level-truncated key slice ([L digits][2][L+1 limbs], special last) gives the same result."""
    ch = small
    L = 4
    key = ch.rand_key()
    trunc = np.concatenate([key[:L, :, :L], key[:L, :, -1:]], axis=2).copy()
    ct, target = ch.rand(2, L, ch.n), ch.rand(L, ch.n)
    got = ch.down(ch.eng.switch_key(ch.up(ct), ch.up(target), ch.up(trunc)))
    assert np.array_equal(got, ch.oc.switch_key(ct, target, key))


@pytest.mark.parametrize("L", [51, 53])
def test_switch_key_many_47bit_digits(L):
    """More digits than the lazy FP64 key MAC can sum exactly (1.25 L q >= 2^53 for q ~ 2^46.9,
    L >= 52): the kernel must fall back to reducing sums (csrc/ntt.h k_ks_row_mac)."""
    ch = Chain(12, [47] * (L + 1), seed=L)
    assert all(q < (1 << 47) and q > (1 << 46) * 1.8 for q in ch.moduli)
    key = ch.rand_key()
    ct, target = ch.rand(2, L, ch.n), ch.rand(L, ch.n)
    got = ch.down(ch.eng.switch_key(ch.up(ct), ch.up(target), ch.up(key)))
    assert np.array_equal(got, ch.oc.switch_key(ct, target, key))
    a, b = ch.rand(2, L, ch.n), ch.rand(2, L, ch.n)
    got = ch.down(ch.eng.hmult(ch.up(a), ch.up(b), ch.up(key)))
    assert np.array_equal(got, ch.oc.hmult(a, b, key))


def test_relinearize(small):
    ch = small
    L = 6
    key = ch.rand_key()
    ct3 = ch.rand(3, L, ch.n)
    t = ch.up(ct3)
    ch.eng.relinearize(t, ch.up(key))
    got = ch.down(t)[:2]
    assert np.array_equal(got, ch.oc.relinearize(ct3, key))


@pytest.mark.parametrize("step", [1, -1, 3, 100, 0])
def test_rotate_vector(small, step):
    """apply_galois_inplace with elt = get_elt_from_step(step) (0 -> conjugation 2N-1)."""
    ch = small
    L = 5
    elt = mhe.galois_elt_from_step(ch.log_n, step)
    assert elt == O.galois_elt_from_step(ch.n, step)
    key = ch.rand_key()
    ct = ch.rand(2, L, ch.n)
    want = ch.oc.apply_galois(ct, elt, key)
    src = ch.up(ct)
    got_to = ch.down(ch.eng.apply_galois_to(src, elt, ch.up(key)))  # out of place: input untouched
    assert np.array_equal(got_to, want)
    assert np.array_equal(ch.down(src), ct)
    got = ch.down(ch.eng.apply_galois(src, elt, ch.up(key)))
    assert np.array_equal(got, want)


def test_apply_galois_ntt_permutation(small):
    ch = small
    a = ch.rand(2, 3, ch.n)
    for elt in (3, 5, 25, 2 * ch.n - 1):
        got = ch.down(ch.eng.permute_galois(ch.up(a), elt))
        want = O.apply_galois_ntt(a.reshape(-1, ch.n), ch.log_n, elt).reshape(a.shape)
        assert np.array_equal(got, want)


def test_mod_switch_drop_to_next(small):
    ch = small
    ct = ch.rand(2, 5, ch.n)
    got = ch.down(ch.eng.mod_switch_drop(ch.up(ct)))
    assert np.array_equal(got, ct[:, :4])
    # in place (out == in): components are compacted downwards
    for size in (2, 3):
        ct = ch.rand(size, 7, ch.n)
        buf = ch.up(ct)
        ch.eng.mod_switch_drop(buf, out=buf)
        flat = ch.down(buf).reshape(-1)[: size * 6 * ch.n].reshape(size, 6, ch.n)
        assert np.array_equal(flat, ct[:, :6])


@pytest.mark.parametrize("L", [1, 3, 8])
def test_modraise(small, L):
    """Bootstrapper::modraise_inplace lift (Bootstrapper.cpp:2894-2948): centered lift of a q_0
    polynomial to L primes; edge coefficients 0, q0/2, q0/2+1, q0-1 included."""
    ch = small
    q0 = ch.moduli[0]
    x = ch.rand(2, 1, ch.n)
    x[0, 0, :4] = [0, q0 >> 1, (q0 >> 1) + 1, q0 - 1]
    got = ch.down(ch.eng.modraise(ch.up(x), L))
    assert np.array_equal(got, ch.oc.modraise(x, L))


def test_hmult_small(small):
    ch = small
    L = ch.K - 1
    key = ch.rand_key()
    a, b = ch.rand(2, L, ch.n), ch.rand(2, L, ch.n)
    got = ch.down(ch.eng.hmult(ch.up(a), ch.up(b), ch.up(key)))
    assert np.array_equal(got, ch.oc.hmult(a, b, key))


@pytest.mark.parametrize("fmt", [1, 2], ids=["doubles", "pack48"])
def test_prepared_key_bit_exact(small, fmt):
    """mhe_key_prepare_as, both engine key formats -- 1: the residues of primes below 2^51 as doubles
    (-0.0 for a zero); 2: 48-bit planes and a tag word for primes below 2^48 -- leaves every key
    switch bit-identical (full and level-truncated keys, switch / relinearize / rotate / HMult),
    and mhe_key_unprepare restores SEAL's layout word for word."""
    ch = small
    key = ch.rand_key()
    key[0, 0, 1, 5] = 0  # a zero residue: -0.0 as a double
    dkey = ch.up(key)
    ch.eng.key_prepare(dkey, fmt)
    assert ch.eng.key_format(dkey) == fmt
    packed = ch.down(dkey)
    if fmt == 1:
        assert all(q < (1 << 51) for q in ch.moduli)  # every limb of this chain is converted
        want = key.astype(np.float64).view(np.uint64).copy()
        want[key == 0] = 0x8000000000000000
        assert np.array_equal(packed, want)
        assert (packed >= (1 << 61)).all()  # no residue of a SEAL key reaches 2^61
    else:
        assert np.array_equal(packed[:, :, 0], key[:, :, 0]) and np.array_equal(packed[:, :, -1], key[:, :, -1])  # 51-bit
        lo = packed[:, :, 1].view(np.uint32)[..., : ch.n]
        hi = packed[:, :, 1].view(np.uint16)[..., 2 * ch.n: 3 * ch.n]
        assert np.array_equal(lo.astype(np.uint64) | (hi.astype(np.uint64) << 32), key[:, :, 1])
        assert (packed[:, :, 1, -1] == 0xF0E1D2C3B4A59687).all()
    for L in (1, 5, ch.K - 1):
        ct, target = ch.rand(2, L, ch.n), ch.rand(L, ch.n)
        got = ch.down(ch.eng.switch_key(ch.up(ct), ch.up(target), dkey))
        assert np.array_equal(got, ch.oc.switch_key(ct, target, key)), L
    L = ch.K - 1
    a, b = ch.rand(2, L, ch.n), ch.rand(2, L, ch.n)
    assert np.array_equal(ch.down(ch.eng.hmult(ch.up(a), ch.up(b), dkey)), ch.oc.hmult(a, b, key))
    elt = mhe.galois_elt_from_step(ch.log_n, 3)
    ct = ch.rand(2, 5, ch.n)
    assert np.array_equal(ch.down(ch.eng.apply_galois_to(ch.up(ct), elt, dkey)), ch.oc.apply_galois(ct, elt, key))
    with pytest.raises(mhe.MheError):
        ch.eng.key_prepare(dkey)  # already prepared
    ch.eng.key_unprepare(dkey)
    assert np.array_equal(ch.down(dkey), key)
    # a level-truncated slice, prepared on its own
    Lt = 4
    trunc = np.concatenate([key[:Lt, :, :Lt], key[:Lt, :, -1:]], axis=2).copy()
    dt = ch.eng.key_prepare(ch.up(trunc), fmt)
    ct, target = ch.rand(2, Lt, ch.n), ch.rand(Lt, ch.n)
    got = ch.down(ch.eng.switch_key(ch.up(ct), ch.up(target), dt))
    assert np.array_equal(got, ch.oc.switch_key(ct, target, key))
    ch.eng.key_unprepare(dt)
    assert np.array_equal(ch.down(dt), trunc)


def test_prepared_key_errors_and_noop():
    """Unpreparing a SEAL-layout key fails with SEAL-style argument errors; on a chain with no
    prime below 2^51 (integer kernels) preparation leaves the key as it is (nothing to convert) and
    switches still match."""
    ch = Chain(12, [60] * 5, seed=11)
    key = ch.rand_key()
    dkey = ch.up(key)
    assert not ch.eng.key_is_prepared(dkey)
    with pytest.raises(mhe.MheError):
        ch.eng.key_unprepare(dkey)
    ch.eng.key_prepare(dkey)
    assert np.array_equal(ch.down(dkey), key) and not ch.eng.key_is_prepared(dkey)
    ct, target = ch.rand(2, 4, ch.n), ch.rand(4, ch.n)
    assert np.array_equal(ch.down(ch.eng.switch_key(ch.up(ct), ch.up(target), dkey)),
                          ch.oc.switch_key(ct, target, key))


def test_errors_are_reported(small):
    ch = small
    key = ch.up(ch.rand_key())
    ct = ch.up(ch.rand(2, 1, ch.n))
    with pytest.raises(mhe.MheError, match="end of modulus switching chain"):
        ch.eng.rescale_to_next(ct)
    with pytest.raises(mhe.MheError, match="Galois element is not valid"):
        ch.eng.permute_galois(ch.up(ch.rand(1, 2, ch.n)), 4)
    too_many = ch.up(ch.rand(2, ch.K, ch.n))  # K limbs > K-1 data limbs
    with pytest.raises(mhe.MheError):
        ch.eng.switch_key(too_many, too_many[0], key)


# ------------------------------------------------------------ decryptable end-to-end
def test_CKKSEncryptMultiplyRelinRescaleDecrypt_small():
    """Mirror of tests/seal/evaluator.cpp:2314 on the GPU: Enc(x)*Enc(x) -> relin -> rescale
    decrypts to x^2 (SURVEY.md §8(d) input kind (ii))."""
    log_n = 13
    moduli = O.coeff_modulus_create(1 << log_n, [51, 46, 46, 46, 51])
    oc = O.Context(log_n, moduli)
    eng = mhe.Engine(log_n, moduli)
    keys = H.keygen(oc, seed=11, hw=64)
    L, scale = 4, 2.0 ** 46
    x = 0.5 * np.cos(2 * np.pi * np.arange((1 << log_n) // 2) / 1024)
    ct = H.encrypt(oc, keys, H.encode(oc, x, scale, L), L)
    out = mhe.Engine.to_host(eng.hmult(eng.to_device(ct), eng.to_device(ct), eng.to_device(keys.relin)))
    assert np.array_equal(out, oc.hmult(ct, ct, keys.relin))
    dec = H.decode(oc, H.decrypt(oc, keys, out), scale * scale / moduli[L - 1])
    assert np.abs(dec - x * x).max() < 1e-6


def test_CKKSEncryptRotateDecrypt_small():
    """Mirror of tests/seal/evaluator.cpp:3100: rotate_vector by k shifts slots left by k."""
    log_n = 12
    moduli = O.coeff_modulus_create(1 << log_n, [51, 46, 46, 51])
    oc = O.Context(log_n, moduli)
    eng = mhe.Engine(log_n, moduli)
    keys = H.keygen(oc, seed=5, hw=64)
    L, scale = 3, 2.0 ** 40
    x = np.random.default_rng(3).uniform(-1, 1, size=(1 << log_n) // 2)
    ct = H.encrypt(oc, keys, H.encode(oc, x, scale, L), L)
    for step in (1, 7, -2):
        elt = mhe.galois_elt_from_step(log_n, step)
        gk = H.galois_key(oc, keys, elt)
        out = mhe.Engine.to_host(eng.apply_galois(eng.to_device(ct), elt, eng.to_device(gk)))
        dec = H.decode(oc, H.decrypt(oc, keys, out), scale)
        assert np.abs(dec - np.roll(x, -step)).max() < 1e-5


# ------------------------------------------------------------------- full size (C2)
@pytest.mark.slow
def test_hmult_c2_full_bit_exact(c2):
    """Config 2 workload (N=2^16, 44 data limbs + special): GPU HMult is
    bit-identical to the oracle on uniform residues and a random relin key."""
    ch = c2
    L = ch.K - 1
    key = ch.rand_key()
    a, b = ch.rand(2, L, ch.n), ch.rand(2, L, ch.n)
    got = ch.down(ch.eng.hmult(ch.up(a), ch.up(b), ch.up(key)))
    want = ch.oc.hmult(a, b, key)
    assert np.array_equal(got, want)


@pytest.mark.slow
def test_hmult_c2_prepared_key_bit_exact(c2):
    """The bench's key format (mhe_key_prepare) at the C2 size: HMult bit-identical to the oracle."""
    ch = c2
    L = ch.K - 1
    key = ch.rand_key()
    a, b = ch.rand(2, L, ch.n), ch.rand(2, L, ch.n)
    dkey = ch.eng.key_prepare(ch.up(key))
    got = ch.down(ch.eng.hmult(ch.up(a), ch.up(b), dkey))
    assert np.array_equal(got, ch.oc.hmult(a, b, key))


@pytest.mark.slow
def test_rotate_c2_full_bit_exact(c2):
    ch = c2
    L = ch.K - 1
    key = ch.rand_key()
    ct = ch.rand(2, L, ch.n)
    elt = mhe.galois_elt_from_step(16, 5)
    want = ch.oc.apply_galois(ct, elt, key)
    src = ch.up(ct)
    got_to = ch.down(ch.eng.apply_galois_to(src, elt, ch.up(key)))  # out of place: input untouched
    assert np.array_equal(got_to, want)
    assert np.array_equal(ch.down(src), ct)
    got = ch.down(ch.eng.apply_galois(src, elt, ch.up(key)))
    assert np.array_equal(got, want)


@pytest.mark.slow
def test_ntt_roundtrip_c2_all_limbs(c2):
    """Size-independent property at full size: INTT(NTT(x)) == x for all 45 limbs, 2 polys."""
    ch = c2
    x = ch.rand(2, ch.K, ch.n)
    t = ch.up(x)
    ch.eng.ntt_forward(t)  # inverse inputs must be < 2q (dwthandler.h:202-233), as in SEAL
    ch.eng.ntt_inverse(t)
    assert np.array_equal(ch.down(t), x)


@pytest.mark.slow
@pytest.mark.parametrize("bits", [RESNET_BITS, GPT2_BITS], ids=["resnet31", "gpt2_60bit_special"])
def test_hmult_reference_chains(bits):
    """The ResNet (31+1) and GPT-2 (36+1, 60-bit special) chains at N=2^16, at a reduced
    level (8 limbs) so the oracle stays in seconds; the key is the full key-level layout."""
    ch = Chain(16, bits, seed=9)
    L = 8
    key = ch.rand_key()
    a, b = ch.rand(2, L, ch.n), ch.rand(2, L, ch.n)
    got = ch.down(ch.eng.hmult(ch.up(a), ch.up(b), ch.up(key)))
    assert np.array_equal(got, ch.oc.hmult(a, b, key))


# ------------------------------------------------------ fused key-switch path (MHE_KS_FUSED)
@pytest.fixture(scope="module")
def fused_engines():
    import os

    old = os.environ.get("MHE_KS_FUSED")
    os.environ["MHE_KS_FUSED"] = "1"
    try:
        small_ch = Chain(12, SMALL_BITS, seed=21)
        full_ch = Chain(16, SMALL_BITS + [51] * 8, seed=22)
    finally:
        if old is None:
            del os.environ["MHE_KS_FUSED"]
        else:
            os.environ["MHE_KS_FUSED"] = old
    return small_ch, full_ch


@pytest.mark.parametrize("L", [1, 3, 7])
def test_switch_key_fused(fused_engines, L):
    ch = fused_engines[0]
    key = ch.rand_key()
    ct, target = ch.rand(2, L, ch.n), ch.rand(L, ch.n)
    got = ch.down(ch.eng.switch_key(ch.up(ct), ch.up(target), ch.up(key)))
    assert np.array_equal(got, ch.oc.switch_key(ct, target, key))


@pytest.mark.slow
def test_hmult_fused_n16(fused_engines):
    ch = fused_engines[1]
    L = ch.K - 1
    key = ch.rand_key()
    a, b = ch.rand(2, L, ch.n), ch.rand(2, L, ch.n)
    got = ch.down(ch.eng.hmult(ch.up(a), ch.up(b), ch.up(key)))
    assert np.array_equal(got, ch.oc.hmult(a, b, key))


# ------------------------------------------- every arithmetic / scheduling variant, bit-exact
ENGINE_VARIANTS = [
    {"MHE_FP": "0"},                                  # integer Harvey/Shoup butterflies everywhere
    {"MHE_FP": "0", "MHE_KS_FUSED": "0"},             # integer, unfused row pass + k_ks_mac
    {"MHE_KS_FUSED": "0"},                            # FP64, unfused
    {"MHE_KS_COLGROUPS": "0"},                        # fused, one column-pass job per (I, J)
    {"MHE_KS_COLGROUPS": "1"},                        # digit-major column pass, one output-prime group
    {"MHE_KS_COLGROUPS": "3", "MHE_KS_SHARE": "0"},   # three groups
    {"MHE_FP": "0", "MHE_KS_COLGROUPS": "2"},
    {"MHE_HMULT_FUSED": "0"},                         # HMult: separate ModDown and rescale
]


def _variant_chain(env, seed):
    import os

    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return Chain(12, SMALL_BITS, seed=seed)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.mark.parametrize("variant", range(len(ENGINE_VARIANTS)))
def test_engine_variants_bit_exact(variant):
    ch = _variant_chain(ENGINE_VARIANTS[variant], 60 + variant)
    key = ch.rand_key()
    for L in (1, 3, ch.K - 1):
        ct, target = ch.rand(2, L, ch.n), ch.rand(L, ch.n)
        got = ch.down(ch.eng.switch_key(ch.up(ct), ch.up(target), ch.up(key)))
        assert np.array_equal(got, ch.oc.switch_key(ct, target, key)), (ENGINE_VARIANTS[variant], L)
    L = ch.K - 1
    a, b = ch.rand(2, L, ch.n), ch.rand(2, L, ch.n)
    got = ch.down(ch.eng.hmult(ch.up(a), ch.up(b), ch.up(key)))
    assert np.array_equal(got, ch.oc.hmult(a, b, key))
    x = ch.rand(2, L, ch.n)
    assert np.array_equal(ch.down(ch.eng.rescale_to_next(ch.up(x))), ch.oc.rescale(x))
    assert np.array_equal(ch.down(ch.eng.ntt_forward(ch.up(x))), ch.oc.ntt(x, O.NTT_FWD))
    assert np.array_equal(ch.down(ch.eng.ntt_inverse(ch.up(x))), ch.oc.ntt(x, O.NTT_INV))


# ------------------------------ n = 2^16 variants: packed intermediate, fused ModDown / galois
# The 48-bit ModUp intermediate (ntt.h tile16) only exists at n = 2^16 for output primes < 2^48,
# so these run on the 7+1-prime chain at log n = 16 (four 46-bit primes): the integer path with
# packing, and each fusion switched off, all against the oracle word for word.
N16_VARIANTS = [
    {},                                                # defaults: FP64, packed, fused
    {"MHE_FP": "0"},                                   # integer butterflies + packed intermediate
    {"MHE_KS_PACK": "0"},                              # 64-bit intermediate
    {"MHE_ICOL_FUSED": "0", "MHE_GALOIS_FUSED": "0"},  # separate inverse column pass, SEAL's galois order
    {"MHE_ICOL_FUSED": "1", "MHE_HMULT_FUSED": "0"},   # fused inverse column pass in the plain ModDown
]


@pytest.mark.parametrize("variant", range(len(N16_VARIANTS)))
def test_n16_variants_bit_exact(variant):
    import os

    env = N16_VARIANTS[variant]
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        ch = Chain(16, SMALL_BITS, seed=70 + variant)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    key = ch.rand_key()
    for L in (2, ch.K - 1):
        ct, target = ch.rand(2, L, ch.n), ch.rand(L, ch.n)
        got = ch.down(ch.eng.switch_key(ch.up(ct), ch.up(target), ch.up(key)))
        assert np.array_equal(got, ch.oc.switch_key(ct, target, key)), (env, L)
    L = ch.K - 1
    a, b = ch.rand(2, L, ch.n), ch.rand(2, L, ch.n)
    assert np.array_equal(ch.down(ch.eng.hmult(ch.up(a), ch.up(b), ch.up(key))), ch.oc.hmult(a, b, key)), env
    x = ch.rand(2, L, ch.n)
    assert np.array_equal(ch.down(ch.eng.rescale_to_next(ch.up(x))), ch.oc.rescale(x)), env
    elt = mhe.galois_elt_from_step(16, 3)
    want = ch.oc.apply_galois(x, elt, key)
    assert np.array_equal(ch.down(ch.eng.apply_galois_to(ch.up(x), elt, ch.up(key))), want), env
    assert np.array_equal(ch.down(ch.eng.apply_galois(ch.up(x), elt, ch.up(key))), want), env


# ----------------------------------------------------------------- CKKS encode (A13, A14)
@pytest.mark.parametrize("kind", ["real", "complex", "partial"])
def test_ckks_encode_bit_exact(small, kind):
    """CKKSEncoder::encode on the engine == the oracle restatement, bit for bit."""
    ch = small
    rng = np.random.default_rng(40)
    if kind == "real":
        v = rng.uniform(-1, 1, ch.n // 2)
    elif kind == "complex":
        v = rng.uniform(-1, 1, ch.n // 2) + 1j * rng.uniform(-1, 1, ch.n // 2)
    else:
        v = rng.uniform(-4, 4, 37)
    L = ch.K - 1
    got = ch.down(ch.eng.encode(v, 2.0 ** 46, L))
    assert np.array_equal(got, ch.oc.encode(v, 2.0 ** 46, L))


@pytest.mark.parametrize("scale", [2.0 ** 20, 2.0 ** 70, 2.0 ** 140])
def test_ckks_encode_wide_coefficients(small, scale):
    """<=64-bit, 128-bit and multi-word coefficient paths (ckks.h:560-628)."""
    ch = small
    v = np.random.default_rng(41).uniform(-1, 1, ch.n // 2)
    L = ch.K - 1
    got = ch.down(ch.eng.encode(v, scale, L))
    assert np.array_equal(got, ch.oc.encode(v, scale, L))


def test_ckks_encode_scalar(small):
    ch = small
    for value, scale in [(0.5, 2.0 ** 40), (-3.25, 2.0 ** 46), (1.0, 2.0 ** 90), (0.0, 2.0 ** 30)]:
        assert ch.eng.encode_scalar(value, scale, ch.K - 1) == ch.oc.encode_scalar(value, scale, ch.K - 1)


def test_ckks_encode_errors(small):
    ch = small
    with pytest.raises(mhe.MheError, match="scale out of bounds"):
        ch.eng.encode([1.0], 2.0 ** 400, 2)
    with pytest.raises(mhe.MheError, match="values_size is too large"):
        ch.eng.encode(np.zeros(ch.n), 2.0 ** 20, 2)


@pytest.mark.slow
def test_ckks_encode_c2_full(c2):
    ch = c2
    v = np.random.default_rng(42).uniform(-1, 1, ch.n // 2) * np.cos(np.arange(ch.n // 2))
    got = ch.down(ch.eng.encode(v, 2.0 ** 46, ch.K - 1))
    assert np.array_equal(got, ch.oc.encode(v, 2.0 ** 46, ch.K - 1))


def test_ckks_encode_at_first_level_bound(small):
    """encode(values, scale, plain) + mod_switch_to_inplace(plain, parms_id) (evaluator.cpp:
    287-310) == encode directly at the lower level with the first level's size checks."""
    ch = small
    v = np.random.default_rng(43).uniform(-1, 1, ch.n // 2)
    full = ch.oc.encode(v, 2.0 ** 46, ch.K - 1)
    got = ch.down(ch.eng.encode(v, 2.0 ** 46, 2, bound_limbs=ch.K - 1))
    assert np.array_equal(got, full[:2])
    # 2^110 * |v| is too wide for 2 limbs (~97 bits) but fine against the first level
    big = ch.oc.encode(v, 2.0 ** 110, ch.K - 1)
    got = ch.down(ch.eng.encode(v, 2.0 ** 110, 2, bound_limbs=ch.K - 1))
    assert np.array_equal(got, big[:2])
    with pytest.raises(mhe.MheError, match="too large|out of bounds"):
        ch.eng.encode(v, 2.0 ** 110, 2)
    assert ch.eng.encode_scalar(0.75, 2.0 ** 110, 2, bound_limbs=ch.K - 1) == \
        ch.oc.encode_scalar(0.75, 2.0 ** 110, ch.K - 1)[:2]


# ----------------------------------------------------------------- CKKS decode
@pytest.mark.parametrize("limbs,scale", [(1, 2.0 ** 30), (3, 2.0 ** 46), (7, 2.0 ** 100)])
def test_ckks_decode_bit_exact(small, limbs, scale):
    """CKKSEncoder::decode on the engine == the oracle restatement, double for double."""
    ch = small
    rng = np.random.default_rng(44 + limbs)
    z = rng.uniform(-1, 1, ch.n // 2) + 1j * rng.uniform(-1, 1, ch.n // 2)
    pt = ch.oc.encode(z, scale, limbs)
    got = ch.eng.decode(ch.up(pt), scale)
    ref = ch.oc.decode(pt, scale)
    assert np.array_equal(got, ref)
    assert np.abs(got - z).max() < 1e-5


def test_ckks_decode_sparse(small):
    ch = small
    pt = ch.rand(3, ch.n)  # arbitrary plaintext (not a valid encoding): exercises every word path
    for sparse in (1, 16, ch.n // 2):
        got = ch.eng.decode(ch.up(pt), 2.0 ** 40, sparse_slots=sparse)
        assert np.array_equal(got, ch.oc.decode(pt, 2.0 ** 40, sparse_slots=sparse))


@pytest.mark.slow
def test_ckks_decode_c2_full(c2):
    ch = c2
    v = np.random.default_rng(45).uniform(-1, 1, ch.n // 2) + 1j * np.random.default_rng(46).uniform(-1, 1, ch.n // 2)
    pt = ch.oc.encode(v, 2.0 ** 46, ch.K - 1)
    got = ch.eng.decode(ch.up(pt), 2.0 ** 46)
    assert np.array_equal(got, ch.oc.decode(pt, 2.0 ** 46))
    assert np.abs(got - v).max() < 1e-6


# ------------------------------------------------------ extreme residues (FP64 bounds)
@pytest.mark.parametrize("bits", [[51] * 8, [51, 46, 46, 51, 46, 51, 51, 51]], ids=["all51", "mixed"])
@pytest.mark.parametrize("fill", ["max", "zero", "alternating", "sparse_max"])
def test_extreme_residues_bit_exact(bits, fill):
    """The exact-FP64 paths (fparith.h: the lazy butterflies, the key MAC, the ModDown / rescale
    lifts and epilogues, the 2^52-offset conversions) at their bounds: every residue q-1, every
    residue 0, alternating 0 / q-1, and mostly-0 with q-1 spikes -- in the ciphertexts, the target
    and the key -- on chains whose primes sit just below 2^51.  HMult, switch_key, rotation and
    rescale must equal the oracle word for word."""
    ch = Chain(12, bits, seed=99)
    L, n, K = ch.K - 1, ch.n, ch.K
    q = np.array(ch.moduli, np.uint64)

    def filled(shape, limbs):
        out = np.empty(shape, np.uint64)
        for l in range(limbs):
            qm1 = np.uint64(int(q[l]) - 1)
            if fill == "max":
                v = np.full(shape[:-2] + (n,), qm1)
            elif fill == "zero":
                v = np.zeros(shape[:-2] + (n,), np.uint64)
            elif fill == "alternating":
                v = np.where(np.arange(n) % 2 == 0, qm1, np.uint64(0)) * np.ones(shape[:-2] + (1,), np.uint64)
            else:
                v = np.where(ch.rng.random(shape[:-2] + (n,)) < 0.01, qm1, np.uint64(0)).astype(np.uint64)
            out[..., l, :] = v
        return out

    a, b = filled((2, L, n), L), filled((2, L, n), L)
    key = np.empty((L, 2, K, n), np.uint64)
    for l in range(K):
        key[:, :, l, :] = np.uint64(int(q[l]) - 1) if fill != "zero" else np.uint64(0)
    dkey = ch.up(key)
    assert np.array_equal(ch.down(ch.eng.hmult(ch.up(a), ch.up(b), dkey)), ch.oc.hmult(a, b, key))
    tgt = filled((L, n), L)
    assert np.array_equal(ch.down(ch.eng.switch_key(ch.up(a), ch.up(tgt), dkey)), ch.oc.switch_key(a, tgt, key))
    elt = mhe.galois_elt_from_step(ch.log_n, 3)
    assert np.array_equal(ch.down(ch.eng.apply_galois_to(ch.up(a), elt, dkey)), ch.oc.apply_galois(a, elt, key))
    assert np.array_equal(ch.down(ch.eng.rescale_to_next(ch.up(a))), ch.oc.rescale(a))
    assert np.array_equal(ch.down(ch.eng.ntt_forward(ch.up(a))), ch.oc.ntt(a, O.NTT_FWD))


MIXED_BITS = [49, 46, 46, 46, 49, 60]  # GPT-2-shaped: data primes < 2^51, a 60-bit special prime


@pytest.mark.parametrize("log_n", [12, 16])
def test_mixed_fp_integer_key_switch(log_n):
    """GPT-2-shaped chain (every data prime < 2^51, special prime 60-bit): the ModUp column pass and
    the fused row-pass MAC run FP64 per output prime below 2^51 and integer for the special prime
    (NttMode fp = 2, MHE_KS_MIX); key switch, HMult and a rotation equal the oracle at every level."""
    ch = Chain(log_n, MIXED_BITS, seed=70 + log_n)
    key = ch.rand_key()
    for L in (1, 3, ch.K - 1):
        ct, target = ch.rand(2, L, ch.n), ch.rand(L, ch.n)
        got = ch.down(ch.eng.switch_key(ch.up(ct), ch.up(target), ch.up(key)))
        assert np.array_equal(got, ch.oc.switch_key(ct, target, key)), L
    L = ch.K - 1
    a, b = ch.rand(2, L, ch.n), ch.rand(2, L, ch.n)
    got = ch.down(ch.eng.hmult(ch.up(a), ch.up(b), ch.up(key)))
    assert np.array_equal(got, ch.oc.hmult(a, b, key))
    elt = mhe.galois_elt_from_step(log_n, 3)
    x = ch.rand(2, L, ch.n)
    got = ch.down(ch.eng.apply_galois(ch.up(x), elt, ch.up(key)))
    assert np.array_equal(got, ch.oc.apply_galois(x, elt, key))
