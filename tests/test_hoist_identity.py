"""The identity behind hoisted rotations (fhe-gpt-2_amd/csrc/hoist.h), checked on the CPU with the
oracle's NTT and Galois permutation (SEAL/util/ntt.cpp, util/galois.cpp:18-51, 192-218).

SEAL rotates a ciphertext by permuting its NTT slots, then key-switches c1: INTT of each limb J
(canonical a^g_J in [0, q_J)), lift to every key prime p_I, NTT (evaluator.cpp:2351-2408).  The engine
lifts and transforms the UNROTATED digit once (D_{I,J} = NTT_{p_I}(a_J mod p_I)) and, per rotation,
reads it permuted and adds (q_J mod p_I) times the NTT of the rotation's negation mask:
    NTT_{p_I}(a^g_J mod p_I) == D_{I,J}[pi_g] + (q_J mod p_I) NTT_{p_I}(mask_g)
for every a_J without a zero coefficient at a slot k >= 1 -- and NOT for one that has (SEAL keeps 0,
not q_J, where the zero is negated), which is why the engine scans for zeros and sends such inputs down
the classic path (tests/test_gpu_batch.py checks both on the GPU)."""
import numpy as np
import pytest

import oracle as O

LOG_N = 10
N = 1 << LOG_N


def negmask(elt):
    """Coefficient-form 0/1 mask: slot t mod N of X^(k g) where k g mod 2N >= N (the moved coefficient
    is negated)."""
    m = np.zeros(N, np.uint64)
    for k in range(N):
        t = (k * elt) % (2 * N)
        m[t % N] = 1 if t >= N else 0
    return m


def lifted_ntt(a, qj, p):
    """NTT_p(a mod p) of a canonical residue vector mod qj (the ModUp of one digit)."""
    return O.ntt(np.asarray(a, np.uint64) % np.uint64(p), LOG_N, p)


@pytest.fixture(scope="module")
def primes():
    return [int(q) for q in O.coeff_modulus_create(N, [46, 51, 46, 51])]


@pytest.mark.parametrize("step", [1, 5, -3, 100, 0])
def test_hoisted_digit_equals_rotated_digit(primes, step):
    rng = np.random.default_rng(7 + step)
    qj = primes[0]
    a = rng.integers(1, qj, N, dtype=np.uint64)  # no zero coefficient
    c1 = O.ntt(a, LOG_N, qj)  # the NTT-form limb J of c1
    elt = O.galois_elt_from_step(N, step) if step else 2 * N - 1  # step 0: the conjugation
    table = O.galois_table_ntt(LOG_N, elt)
    a_rot = O.ntt(O.apply_galois_ntt(c1, LOG_N, elt), LOG_N, qj, O.NTT_INV)  # SEAL's a^g_J, canonical
    for p in primes[1:]:
        want = lifted_ntt(a_rot, qj, p)
        D = lifted_ntt(a, qj, p)
        M = O.ntt(negmask(elt), LOG_N, p)
        got = (D[table].astype(object) + (qj % p) * M.astype(object)) % p
        assert np.array_equal(np.array(got, np.uint64), want), f"prime {p}"


def test_identity_fails_at_a_negated_zero(primes):
    """A zero coefficient moved to a negated slot stays 0 in SEAL's canonical form, while the identity
    adds q_J there: the two differ, so the engine must not hoist such an input."""
    rng = np.random.default_rng(3)
    qj, p = primes[0], primes[1]
    elt = O.galois_elt_from_step(N, 1)
    m = negmask(elt)
    a = rng.integers(1, qj, N, dtype=np.uint64)
    # the coefficient that lands on a negated slot
    k = next(k for k in range(1, N) if (k * elt) % (2 * N) >= N)
    a[k] = 0
    c1 = O.ntt(a, LOG_N, qj)
    table = O.galois_table_ntt(LOG_N, elt)
    a_rot = O.ntt(O.apply_galois_ntt(c1, LOG_N, elt), LOG_N, qj, O.NTT_INV)
    want = lifted_ntt(a_rot, qj, p)
    got = (lifted_ntt(a, qj, p)[table].astype(object) + (qj % p) * O.ntt(m, LOG_N, p).astype(object)) % p
    assert not np.array_equal(np.array(got, np.uint64), want)
    # ... and exactly by (q_J mod p) times the NTT of that one monomial
    mono = np.zeros(N, np.uint64)
    mono[((k * elt) % (2 * N)) % N] = 1
    fix = (qj % p) * O.ntt(mono, LOG_N, p).astype(object)
    assert np.array_equal(np.array((got - fix) % p, np.uint64), want)
