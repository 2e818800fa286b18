"""ctypes wrapper over oracle/liboracle.so -- the CPU restatement of the reference's
RNS-CKKS evaluator (see mhe_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product path (fhe-gpt-2_amd/).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

u64p = ctypes.POINTER(ctypes.c_uint64)
u32p = ctypes.POINTER(ctypes.c_uint32)


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def build_native(dst_dir):
    """Compile the restatement for the host it runs on (-O3 -march=native; the committed build is
    portable because the .so travels between machines) into dst_dir and load that build instead.
    Used by bench.py's cpu_baseline leg on the GPU box.  Returns the library path."""
    global _LIB_PATH, _lib
    out = os.path.join(dst_dir, "liboracle_native.so")
    subprocess.check_call(["gcc", "-O3", "-march=native", "-fPIC", "-fopenmp", "-ffp-contract=off", "-shared",
                           "-o", out, os.path.join(_HERE, "mhe_oracle.c"), "-lm"])
    _LIB_PATH, _lib = out, None
    return out


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        sig = {
            "or_is_prime": (ctypes.c_int, [ctypes.c_uint64]),
            "or_get_primes": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, u64p]),
            "or_coeff_modulus_create": (ctypes.c_int, [ctypes.c_uint64, ctypes.POINTER(ctypes.c_int), ctypes.c_int, u64p]),
            "or_minimal_primitive_root": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint64]),
            "or_barrett_reduce_64": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint64]),
            "or_barrett_reduce_128": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]),
            "or_multiply_uint_mod": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]),
            "or_shoup_quotient": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint64]),
            "or_multiply_uint_mod_shoup": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]),
            "or_try_invert_uint_mod": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint64, u64p]),
            "or_ntt_root_powers": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint64, u64p, u64p]),
            "or_ntt": (ctypes.c_int, [u64p, ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_int]),
            "or_ctx_create": (ctypes.c_void_p, [ctypes.c_int, u64p, ctypes.c_int]),
            "or_ctx_destroy": (None, [ctypes.c_void_p]),
            "or_ctx_ntt": (None, [ctypes.c_void_p, u64p, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
            "or_ctx_dyadic": (None, [ctypes.c_void_p, u64p, u64p, u64p, ctypes.c_int]),
            "or_ctx_addsub": (None, [ctypes.c_void_p, u64p, u64p, u64p, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
            "or_ctx_ckks_multiply": (None, [ctypes.c_void_p, u64p, u64p, u64p, ctypes.c_int]),
            "or_ctx_ckks_square": (None, [ctypes.c_void_p, u64p, u64p, ctypes.c_int]),
            "or_ctx_switch_key": (ctypes.c_int, [ctypes.c_void_p, u64p, u64p, u64p, ctypes.c_int]),
            "or_ctx_relinearize": (ctypes.c_int, [ctypes.c_void_p, u64p, u64p, ctypes.c_int]),
            "or_ctx_rescale": (ctypes.c_int, [ctypes.c_void_p, u64p, u64p, ctypes.c_int, ctypes.c_int]),
            "or_galois_elt_from_step": (ctypes.c_uint32, [ctypes.c_uint64, ctypes.c_int]),
            "or_galois_table_ntt": (None, [ctypes.c_int, ctypes.c_uint32, u32p]),
            "or_apply_galois_ntt": (None, [u64p, ctypes.c_int, ctypes.c_int, ctypes.c_uint32, u64p]),
            "or_ctx_apply_galois": (ctypes.c_int, [ctypes.c_void_p, u64p, ctypes.c_uint32, u64p, ctypes.c_int]),
            "or_ctx_multiply_plain": (None, [ctypes.c_void_p, u64p, u64p, ctypes.c_int, ctypes.c_int]),
            "or_ctx_hmult": (ctypes.c_int, [ctypes.c_void_p, u64p, u64p, u64p, u64p, ctypes.c_int]),
            "or_ctx_hmult_batch": (ctypes.c_int, [ctypes.c_void_p, u64p, u64p, u64p, u64p, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
            "or_ctx_hmult_batch_cyclic": (ctypes.c_int, [ctypes.c_void_p, u64p, u64p, ctypes.c_int, u64p, u64p, ctypes.c_int,
                                                         ctypes.c_int, ctypes.c_int]),
            "or_encoder_create": (ctypes.c_void_p, [ctypes.c_int]),
            "or_encoder_destroy": (None, [ctypes.c_void_p]),
            "or_ckks_encode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                              ctypes.POINTER(ctypes.c_double), ctypes.c_size_t, ctypes.c_double,
                                              ctypes.c_int, ctypes.c_int, u64p]),
            "or_ckks_encode_scalar": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                                     ctypes.c_int, u64p]),
            "or_ckks_decode_coeffs": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, u64p, ctypes.c_int,
                                                     ctypes.c_double, ctypes.c_int, ctypes.c_size_t,
                                                     ctypes.POINTER(ctypes.c_double)]),
            "or_ckks_decode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, u64p, ctypes.c_int, ctypes.c_double,
                                              ctypes.c_int, ctypes.c_size_t, ctypes.POINTER(ctypes.c_double),
                                              ctypes.POINTER(ctypes.c_double)]),
            "or_blake2xb": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                           ctypes.c_char_p, ctypes.c_size_t]),
            "or_prng_bytes": (None, [u64p, ctypes.c_size_t, ctypes.c_char_p]),
            "or_ctx_sample": (None, [ctypes.c_void_p, u64p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, u64p]),
            "or_ctx_encrypt_zero_symmetric": (None, [ctypes.c_void_p, u64p, u64p, ctypes.c_int, u64p]),
            "or_ctx_encrypt_zero_asymmetric": (None, [ctypes.c_void_p, u64p, u64p, ctypes.c_int, ctypes.c_int, u64p]),
            "or_ctx_keygen_secret": (None, [ctypes.c_void_p, u64p, ctypes.c_size_t, u64p]),
            "or_ctx_kswitch_key": (None, [ctypes.c_void_p, u64p, u64p, u64p, u64p]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _p(a):
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"], (a.dtype, a.flags)
    return a.ctypes.data_as(u64p)


# ---------------------------------------------------------------- SEAL randomness (seal_random.c)
def blake2xb(outlen, data, key):
    """blake2xb(out, outlen, in, inlen, key, keylen) (util/blake2xb.c:143-168)."""
    out = ctypes.create_string_buffer(outlen)
    rc = lib().or_blake2xb(out, outlen, bytes(data), len(data), bytes(key), len(key))
    assert rc == 0
    return out.raw


def _seed(seed):
    s = np.ascontiguousarray(np.array(seed, dtype=np.uint64))
    assert s.shape == (8,)
    return s


def prng_bytes(seed, count):
    """The first `count` bytes of Blake2xbPRNG(seed) (randomgen.cpp:160-195)."""
    s = _seed(seed)
    out = ctypes.create_string_buffer(count)
    lib().or_prng_bytes(_p(s), count, out)
    return out.raw


# ---------------------------------------------------------------- scalar / table helpers
def is_prime(v):
    return bool(lib().or_is_prime(v))


def get_primes(n, bits, count):
    out = np.zeros(count, np.uint64)
    got = lib().or_get_primes(n, bits, count, _p(out))
    return [int(x) for x in out[:got]]


def coeff_modulus_create(n, bit_sizes):
    bs = (ctypes.c_int * len(bit_sizes))(*bit_sizes)
    out = np.zeros(len(bit_sizes), np.uint64)
    if lib().or_coeff_modulus_create(n, bs, len(bit_sizes), _p(out)) != 0:
        raise ValueError("failed to find enough qualifying primes")
    return [int(x) for x in out]


def minimal_primitive_root(degree, q):
    return int(lib().or_minimal_primitive_root(degree, q))


def ntt_root_powers(log_n, q):
    n = 1 << log_n
    r = np.zeros(n, np.uint64)
    ir = np.zeros(n, np.uint64)
    if lib().or_ntt_root_powers(log_n, q, _p(r), _p(ir)):
        raise ValueError("invalid modulus")
    return r, ir


NTT_FWD, NTT_FWD_LAZY, NTT_INV, NTT_INV_LAZY = 0, 1, 2, 3


def ntt(data, log_n, q, mode=NTT_FWD):
    a = np.ascontiguousarray(data, dtype=np.uint64).copy()
    n = 1 << log_n
    assert a.size % n == 0
    if lib().or_ntt(_p(a), log_n, q, a.size // n, mode):
        raise ValueError("invalid modulus")
    return a


def galois_elt_from_step(n, step):
    return int(lib().or_galois_elt_from_step(n, step))


def galois_table_ntt(log_n, elt):
    t = np.zeros(1 << log_n, np.uint32)
    lib().or_galois_table_ntt(log_n, elt, t.ctypes.data_as(u32p))
    return t


def apply_galois_ntt(data, log_n, elt):
    a = np.ascontiguousarray(data, dtype=np.uint64)
    out = np.zeros_like(a)
    limbs = a.size >> log_n
    lib().or_apply_galois_ntt(_p(a), log_n, limbs, elt, _p(out))
    return out


class Context:
    """Key-level modulus chain (data primes then the special prime), like
    SEALContext::key_context_data (context.cpp:422-523)."""

    def __init__(self, log_n, moduli):
        self.log_n = log_n
        self.n = 1 << log_n
        self.moduli = [int(q) for q in moduli]
        self.k = len(self.moduli)
        arr = np.array(self.moduli, np.uint64)
        self._h = lib().or_ctx_create(log_n, _p(arr), self.k)
        if not self._h:
            raise ValueError("invalid modulus chain")

    def __del__(self):
        if getattr(self, "_enc", None):
            lib().or_encoder_destroy(self._enc)
            self._enc = None
        if getattr(self, "_h", None):
            lib().or_ctx_destroy(self._h)
            self._h = None

    def ntt(self, data, mode=NTT_FWD):
        a = np.ascontiguousarray(data, dtype=np.uint64).copy()
        polys, limbs = (1, a.shape[0]) if a.ndim == 2 else a.shape[:2]
        lib().or_ctx_ntt(self._h, _p(a), polys, limbs, mode)
        return a

    def dyadic(self, a, b):
        a = np.ascontiguousarray(a, np.uint64)
        b = np.ascontiguousarray(b, np.uint64)
        out = np.empty_like(a)
        lib().or_ctx_dyadic(self._h, _p(a), _p(b), _p(out), a.shape[-2])
        return out

    def _addsub(self, a, b, op):
        a = np.ascontiguousarray(a, np.uint64)
        b = a if b is None else np.ascontiguousarray(b, np.uint64)
        polys, limbs = (1, a.shape[0]) if a.ndim == 2 else a.shape[:2]
        out = np.empty_like(a)
        lib().or_ctx_addsub(self._h, _p(a), _p(b), _p(out), polys, limbs, op)
        return out

    def add(self, a, b):
        return self._addsub(a, b, 0)

    def sub(self, a, b):
        return self._addsub(a, b, 1)

    def negate(self, a):
        return self._addsub(a, None, 2)

    def multiply(self, a, b):
        L = a.shape[1]
        out = np.empty((3, L, self.n), np.uint64)
        lib().or_ctx_ckks_multiply(self._h, _p(np.ascontiguousarray(a)), _p(np.ascontiguousarray(b)), _p(out), L)
        return out

    def square(self, a):
        L = a.shape[1]
        out = np.empty((3, L, self.n), np.uint64)
        lib().or_ctx_ckks_square(self._h, _p(np.ascontiguousarray(a)), _p(out), L)
        return out

    def switch_key(self, ct, target, key):
        ct = np.ascontiguousarray(ct, np.uint64).copy()
        L = ct.shape[1]
        if lib().or_ctx_switch_key(self._h, _p(ct), _p(np.ascontiguousarray(target, np.uint64)), _p(key), L):
            raise ValueError("switch_key: bad level")
        return ct

    def relinearize(self, ct3, key):
        ct3 = np.ascontiguousarray(ct3, np.uint64).copy()
        L = ct3.shape[1]
        if lib().or_ctx_relinearize(self._h, _p(ct3), _p(key), L):
            raise ValueError("relinearize: bad level")
        return ct3[:2].copy()

    def rescale(self, ct):
        ct = np.ascontiguousarray(ct, np.uint64)
        size, L = ct.shape[:2]
        out = np.empty((size, L - 1, self.n), np.uint64)
        if lib().or_ctx_rescale(self._h, _p(ct), _p(out), size, L):
            raise ValueError("end of modulus switching chain reached")
        return out

    def apply_galois(self, ct, elt, key):
        ct = np.ascontiguousarray(ct, np.uint64).copy()
        if lib().or_ctx_apply_galois(self._h, _p(ct), elt, _p(key), ct.shape[1]):
            raise ValueError("apply_galois: bad level")
        return ct

    def multiply_plain(self, ct, pt):
        ct = np.ascontiguousarray(ct, np.uint64).copy()
        size, L = ct.shape[:2]
        lib().or_ctx_multiply_plain(self._h, _p(ct), _p(np.ascontiguousarray(pt, np.uint64)), size, L)
        return ct

    def modraise(self, ct1, L):
        """Bootstrapper::modraise_inplace lift (ckks_bootstrapping/Bootstrapper.cpp:2929-2945):
        poly_dest[i] = x % q; if x > q0/2: += q - q0 % q, conditional subtract.  ct1 is the
        coefficient-form [size][1][n] polynomial mod q0; returns [size][L][n] (coefficient form)."""
        import numpy as np

        q0 = int(self.moduli[0])
        x = np.asarray(ct1[:, 0, :], dtype=np.uint64)
        out = np.empty((x.shape[0], L, x.shape[1]), dtype=np.uint64)
        hi = x > np.uint64(q0 >> 1)
        for j in range(L):
            q = int(self.moduli[j])
            v = x % np.uint64(q)
            mq0 = np.uint64(q - q0 % q)
            w = v + mq0
            w = np.where(w >= np.uint64(q), w - np.uint64(q), w)
            out[:, j, :] = np.where(hi, w, v)
        return out

    def hmult(self, a, b, key):
        L = a.shape[1]
        out = np.empty((2, L - 1, self.n), np.uint64)
        if lib().or_ctx_hmult(self._h, _p(np.ascontiguousarray(a)), _p(np.ascontiguousarray(b)), _p(key), _p(out), L):
            raise ValueError("hmult failed")
        return out

    def total_bits(self, limbs):
        """ContextData::total_coeff_modulus_bit_count of the level with `limbs` primes."""
        p = 1
        for q in self.moduli[:limbs]:
            p *= q
        return p.bit_length()

    def encode(self, values, scale, limbs):
        """CKKSEncoder::encode (ckks.h:457-640) -> NTT-form plaintext [limbs][n]."""
        if not hasattr(self, "_enc"):
            self._enc = lib().or_encoder_create(self.log_n)
        v = np.asarray(values)
        re = np.ascontiguousarray(v.real, np.float64)
        im = np.ascontiguousarray(v.imag, np.float64) if np.iscomplexobj(v) else None
        out = np.zeros((limbs, self.n), np.uint64)
        dp = ctypes.POINTER(ctypes.c_double)
        rc = lib().or_ckks_encode(self._enc, self._h, re.ctypes.data_as(dp), im.ctypes.data_as(dp) if im is not None else None,
                                  re.size, scale, limbs, self.total_bits(limbs), _p(out))
        if rc == -1:
            raise ValueError("scale out of bounds")
        if rc == -2:
            raise ValueError("encoded values are too large")
        return out

    def encode_scalar(self, value, scale, limbs):
        """CKKSEncoder::encode(double) (ckks.cpp:78-200) -> one residue per limb."""
        out = np.zeros(limbs, np.uint64)
        rc = lib().or_ckks_encode_scalar(self._h, value, scale, limbs, self.total_bits(limbs), _p(out))
        if rc:
            raise ValueError("scale out of bounds" if rc == -1 else "encoded value is too large")
        return [int(x) for x in out]

    def decode(self, plain, scale, sparse_slots=0):
        """CKKSEncoder::decode (ckks.h:644-761): NTT-form plaintext [limbs][n] -> complex slots."""
        if not hasattr(self, "_enc"):
            self._enc = lib().or_encoder_create(self.log_n)
        plain = np.ascontiguousarray(plain, np.uint64)
        limbs = plain.shape[0]
        cnt = sparse_slots or self.n // 2
        re = np.zeros(cnt, np.float64)
        im = np.zeros(cnt, np.float64)
        dp = ctypes.POINTER(ctypes.c_double)
        rc = lib().or_ckks_decode(self._enc, self._h, _p(plain), limbs, scale, self.total_bits(limbs), sparse_slots,
                                  re.ctypes.data_as(dp), im.ctypes.data_as(dp))
        if rc:
            raise ValueError("scale out of bounds")
        return re + 1j * im

    def decode_coeffs(self, plain, scale, sparse_slots=0):
        """The doubles decode() feeds to transform_to_rev (ckks.h:715-753)."""
        if not hasattr(self, "_enc"):
            self._enc = lib().or_encoder_create(self.log_n)
        plain = np.ascontiguousarray(plain, np.uint64)
        out = np.zeros(self.n, np.float64)
        rc = lib().or_ckks_decode_coeffs(self._enc, self._h, _p(plain), plain.shape[0], scale,
                                         self.total_bits(plain.shape[0]), sparse_slots,
                                         out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        if rc:
            raise ValueError("scale out of bounds")
        return out

    SAMPLE = {"uniform": 0, "ternary": 1, "sparse_ternary": 2, "cbd": 3}

    def sample(self, seed, kind, limbs, hw=0):
        """[limbs][n] residues of SEAL's sample_poly_<kind>(Blake2xbPRNG(seed)) (rlwe.cpp:21-162)."""
        out = np.zeros((limbs, self.n), np.uint64)
        s = _seed(seed)
        lib().or_ctx_sample(self._h, _p(s), self.SAMPLE[kind], limbs, hw, _p(out))
        return out

    def keygen_secret(self, seed, hw):
        out = np.zeros((self.k, self.n), np.uint64)
        s = _seed(seed)
        lib().or_ctx_keygen_secret(self._h, _p(s), hw, _p(out))
        return out

    def encrypt_zero_symmetric(self, seed, sk, limbs):
        out = np.zeros((2, limbs, self.n), np.uint64)
        s, sk = _seed(seed), np.ascontiguousarray(sk)
        lib().or_ctx_encrypt_zero_symmetric(self._h, _p(s), _p(sk), limbs, _p(out))
        return out

    def encrypt_zero_asymmetric(self, seed, pk, m, L):
        out = np.zeros((2, L, self.n), np.uint64)
        s, pk = _seed(seed), np.ascontiguousarray(pk)
        lib().or_ctx_encrypt_zero_asymmetric(self._h, _p(s), _p(pk), m, L, _p(out))
        return out

    def kswitch_key(self, seed, sk, new_key):
        out = np.zeros((self.k - 1, 2, self.k, self.n), np.uint64)
        s, sk, nk = _seed(seed), np.ascontiguousarray(sk), np.ascontiguousarray(new_key)
        lib().or_ctx_kswitch_key(self._h, _p(s), _p(sk), _p(nk), _p(out))
        return out

    def hmult_batch(self, a, b, key, threads=0):
        """a, b: [B][2][L][n] -> ([B][2][L-1][n], threads used)."""
        B, _, L = a.shape[:3]
        out = np.empty((B, 2, L - 1, self.n), np.uint64)
        used = lib().or_ctx_hmult_batch(self._h, _p(np.ascontiguousarray(a)), _p(np.ascontiguousarray(b)), _p(key),
                                        _p(out), L, B, threads)
        return out, used

    def hmult_batch_cyclic(self, a, b, key, batch, threads, out=None):
        """`batch` independent HMults over the a[i % D], b[i % D] pairs (a, b: [D][2][L][n]) on
        `threads` OpenMP threads; each thread writes its slot of out [threads][2][L-1][n] (pass a
        pre-touched buffer to keep page faults out of a timing).  Returns the threads used."""
        D, _, L = a.shape[:3]
        if out is None:
            out = np.zeros((threads, 2, L - 1, self.n), np.uint64)
        return lib().or_ctx_hmult_batch_cyclic(self._h, _p(np.ascontiguousarray(a)), _p(np.ascontiguousarray(b)), D,
                                               _p(key), _p(out), L, batch, threads)
