"""GPU parity of key generation and encryption with SEAL's randomness (A18).

build/random_test (tests/cpp/random_test.cpp) draws, through the seal:: surface on the GPU, with
a Blake2xbPRNGFactory seeded {1..8}: the secret key (sparse ternary), the public key, the
relinearization key, the step-1 Galois key (full and truncated to 2-limb ciphertexts), public-key
encryptions of zero at the first level and at 2 limbs, and a secret-key encryption of zero.  Each
is compared bit for bit with the oracle's sequential restatement of SEAL (oracle/seal_random.c:
keygenerator.cpp, rlwe.cpp, encryptor.cpp), itself pinned by hashlib (test_seal_random.py).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

SEED = [1, 2, 3, 4, 5, 6, 7, 8]
EXE = os.path.join(ROOT, "build", "random_test")


@pytest.mark.gpu
@pytest.mark.parametrize("log_n,hw,bits", [
    (12, 32, [50, 40, 40, 50]),
    (13, 0, [55, 45, 45, 45, 55]),  # hw 0: ternary secret key (sample_poly_ternary)
])
def test_keys_and_encryptions_match_oracle(tmp_path, log_n, hw, bits):
    if not os.path.exists(EXE):
        pytest.fail("build/random_test missing: run __graft_entry__.build()")
    p = subprocess.run([EXE, str(tmp_path), str(log_n), str(hw)] + [str(b) for b in bits],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    n, K = 1 << log_n, len(bits)
    moduli = O.coeff_modulus_create(n, bits)
    oc = O.Context(log_n, moduli)

    def load(name, shape):
        return np.fromfile(tmp_path / name, dtype=np.uint64).reshape(shape)

    sk = oc.keygen_secret(SEED, hw)
    assert np.array_equal(load("sk.bin", (K, n)), sk)
    pk = oc.encrypt_zero_symmetric(SEED, sk, K)
    assert np.array_equal(load("pk.bin", (2, K, n)), pk)
    relin = oc.kswitch_key(SEED, sk, oc.dyadic(sk, sk))
    assert np.array_equal(load("relin.bin", (K - 1, 2, K, n)), relin)
    rot = O.apply_galois_ntt(sk, log_n, 5)
    gal = oc.kswitch_key(SEED, sk, rot)
    assert np.array_equal(load("galois1.bin", (K - 1, 2, K, n)), gal)
    trunc = np.concatenate([gal[:2, :, :2, :], gal[:2, :, K - 1:, :]], axis=2)
    assert np.array_equal(load("galois1_trunc2.bin", (2, 2, 3, n)), trunc)
    asym = oc.encrypt_zero_asymmetric(SEED, pk, K, K - 1)
    assert np.array_equal(load("asym_first.bin", (2, K - 1, n)), asym)
    asym2 = oc.encrypt_zero_asymmetric(SEED, pk, 3, 2)
    assert np.array_equal(load("asym_l2.bin", (2, 2, n)), asym2)
    sym = oc.encrypt_zero_symmetric(SEED, sk, K - 1)
    assert np.array_equal(load("sym_first.bin", (2, K - 1, n)), sym)
    # sanity: the secret key is sparse ternary of the requested weight
    if hw:
        coeff = oc.ntt(sk, O.NTT_INV)
        nz = (coeff[0] != 0).sum()
        assert nz in (hw, hw - 1)  # index n (SEAL's inclusive range) touches limb 1 only
