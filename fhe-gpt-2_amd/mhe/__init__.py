"""Python binding of libmhe.so (include/mhe.h) for tests and bench.

Thin ctypes layer: one method per C-ABI entry point, named after the SEAL evaluator step it
replaces.  Device memory and streams come from PyTorch (plumbing only); every compute call
goes through the HIP kernels in libmhe.so.  There is no CPU fallback: if the library or the
GPU is missing, construction raises.

Device arrays are torch int64 tensors holding the u64 residue bits ([poly][limb][n]).
"""
import ctypes
import os

import numpy as np

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_DEFAULT_LIB = os.path.join(_PKG, "libmhe.so")
LIB_PATH = os.environ.get("MHE_LIB_PATH") or _DEFAULT_LIB  # override: build experiments
_lib = None

u64p = ctypes.POINTER(ctypes.c_uint64)
vp = ctypes.c_void_p

# name -> (restype, argtypes); mirrors include/mhe.h
SIGNATURES = {
    "mhe_last_error": (ctypes.c_char_p, []),
    "mhe_version": (ctypes.c_int, []),
    "mhe_ctx_create": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.c_int, u64p, ctypes.c_int, ctypes.c_int]),
    "mhe_ctx_destroy": (ctypes.c_int, [vp]),
    "mhe_ctx_reserve": (ctypes.c_int, [vp, ctypes.c_int, vp]),
    "mhe_coeff_modulus_create": (ctypes.c_int, [ctypes.c_uint64, ctypes.POINTER(ctypes.c_int), ctypes.c_int, u64p]),
    "mhe_galois_elt_from_step": (ctypes.c_uint32, [ctypes.c_int, ctypes.c_int]),
    "mhe_malloc": (ctypes.c_int, [vp, ctypes.POINTER(vp), ctypes.c_size_t]),
    "mhe_free": (ctypes.c_int, [vp, vp]),
    "mhe_ctx_set_timing": (ctypes.c_int, [vp, ctypes.c_int]),
    "mhe_kernel_time": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]),
    "mhe_ctx_set_hoist": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int]),
    "mhe_ctx_get_hoist": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "mhe_hoist_stats": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                       ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]),
    "mhe_debug_fail_alloc": (ctypes.c_int, [vp, ctypes.c_int]),
    "mhe_debug_fail_switch": (ctypes.c_int, [vp, ctypes.c_int]),
    "mhe_alloc_stats": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]),
    "mhe_trim": (ctypes.c_int, [vp]),
    "mhe_scratch_bytes": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                         ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int)]),
    "mhe_malloc_async": (ctypes.c_int, [vp, ctypes.POINTER(vp), ctypes.c_size_t, vp]),
    "mhe_free_async": (ctypes.c_int, [vp, vp, vp]),
    "mhe_memcpy_h2d": (ctypes.c_int, [vp, vp, vp, ctypes.c_size_t, vp]),
    "mhe_memcpy_d2h": (ctypes.c_int, [vp, vp, vp, ctypes.c_size_t, vp]),
    "mhe_memcpy_d2d": (ctypes.c_int, [vp, vp, vp, ctypes.c_size_t, vp]),
    "mhe_stream_sync": (ctypes.c_int, [vp, vp]),
    "mhe_stream_wait": (ctypes.c_int, [vp, vp, vp]),
    "mhe_multiply_plain_add": (ctypes.c_int, [vp, vp, vp, vp, ctypes.c_int, ctypes.c_int, vp]),
    "mhe_multiply_plain_sum": (ctypes.c_int, [vp, ctypes.c_int, vp, vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              vp]),
    "mhe_key_traffic": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]),
    "mhe_op_counts": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int, ctypes.c_int]),
    # launch hook (seal::FiberBatch coalesces elementwise launches through it; Python never sets one)
    "mhe_set_launch_hook": (ctypes.c_int, [vp, vp]),
    "mhe_launch_run": (ctypes.c_int, [vp, vp, ctypes.c_int]),
    "mhe_key_prepare": (ctypes.c_int, [vp, vp, ctypes.c_int, ctypes.c_int, vp]),
    "mhe_key_prepare_as": (ctypes.c_int, [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp]),
    "mhe_key_unprepare": (ctypes.c_int, [vp, vp, ctypes.c_int, ctypes.c_int, vp]),
    "mhe_key_is_prepared": (ctypes.c_int, [vp, vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int), vp]),
    "mhe_key_traffic_prepared": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]),
    "mhe_stream_create": (ctypes.c_int, [vp, ctypes.POINTER(vp)]),
    "mhe_stream_destroy": (ctypes.c_int, [vp, vp]),
    "mhe_ntt_forward": (ctypes.c_int, [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp]),
    "mhe_ntt_inverse": (ctypes.c_int, [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp]),
    "mhe_add": (ctypes.c_int, [vp, vp, vp, vp, ctypes.c_int, ctypes.c_int, vp]),
    "mhe_sub": (ctypes.c_int, [vp, vp, vp, vp, ctypes.c_int, ctypes.c_int, vp]),
    "mhe_negate": (ctypes.c_int, [vp, vp, vp, ctypes.c_int, ctypes.c_int, vp]),
    "mhe_multiply_plain": (ctypes.c_int, [vp, vp, vp, vp, ctypes.c_int, ctypes.c_int, vp]),
    "mhe_multiply_scalar": (ctypes.c_int, [vp, vp, u64p, vp, ctypes.c_int, ctypes.c_int, vp]),
    "mhe_add_scalar": (ctypes.c_int, [vp, vp, u64p, vp, ctypes.c_int, ctypes.c_int, vp]),
    "mhe_set_scalar": (ctypes.c_int, [vp, u64p, vp, ctypes.c_int, ctypes.c_int, vp]),
    "mhe_ct_multiply": (ctypes.c_int, [vp, vp, vp, vp, ctypes.c_int, vp]),
    "mhe_ct_square": (ctypes.c_int, [vp, vp, vp, ctypes.c_int, vp]),
    "mhe_switch_key": (ctypes.c_int, [vp, vp, vp, vp, ctypes.c_int, ctypes.c_int, vp]),
    "mhe_relinearize": (ctypes.c_int, [vp, vp, vp, ctypes.c_int, ctypes.c_int, vp]),
    "mhe_apply_galois": (ctypes.c_int, [vp, vp, ctypes.c_uint32, vp, ctypes.c_int, ctypes.c_int, vp]),
    "mhe_apply_galois_to": (ctypes.c_int, [vp, vp, vp, ctypes.c_uint32, vp, ctypes.c_int, ctypes.c_int, vp]),
    "mhe_permute_galois": (ctypes.c_int, [vp, vp, ctypes.c_uint32, vp, ctypes.c_int, ctypes.c_int, vp]),
    "mhe_rescale_to_next": (ctypes.c_int, [vp, vp, vp, ctypes.c_int, ctypes.c_int, vp]),
    "mhe_apply_galois_batch": (ctypes.c_int, [vp, ctypes.c_int, vp, vp, ctypes.POINTER(ctypes.c_uint32), vp,
                                              ctypes.POINTER(ctypes.c_int), ctypes.c_int, vp]),
    "mhe_rescale_batch": (ctypes.c_int, [vp, ctypes.c_int, vp, vp, ctypes.c_int, ctypes.c_int, vp]),
    "mhe_switch_key_batch": (ctypes.c_int, [vp, ctypes.c_int, vp, vp, vp, ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                            vp]),
    "mhe_mod_switch_drop": (ctypes.c_int, [vp, vp, vp, ctypes.c_int, ctypes.c_int, vp]),
    "mhe_modraise": (ctypes.c_int, [vp, vp, vp, ctypes.c_int, ctypes.c_int, vp]),
    "mhe_hmult": (ctypes.c_int, [vp, vp, vp, vp, ctypes.c_int, vp, ctypes.c_int, vp]),
    "mhe_hmult_batch": (ctypes.c_int, [vp, ctypes.c_int, vp, vp, vp, ctypes.c_int, vp, ctypes.c_int, vp]),
    "mhe_encoder_create": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.c_int]),
    "mhe_encoder_destroy": (ctypes.c_int, [vp]),
    "mhe_ckks_encode": (ctypes.c_int, [vp, vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                       ctypes.c_size_t, ctypes.c_double, ctypes.c_int, vp, vp]),
    "mhe_ckks_encode_scalar": (ctypes.c_int, [vp, ctypes.c_double, ctypes.c_double, ctypes.c_int, u64p]),
    "mhe_ckks_encode_at": (ctypes.c_int, [vp, vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                          ctypes.c_size_t, ctypes.c_double, ctypes.c_int, ctypes.c_int, vp, vp]),
    "mhe_ckks_decode": (ctypes.c_int, [vp, vp, vp, ctypes.c_int, ctypes.c_double, ctypes.c_size_t,
                                       ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), vp]),
    "mhe_ckks_encode_scalar_at": (ctypes.c_int, [vp, ctypes.c_double, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                                 u64p]),
    "mhe_prng_uniform_bulk": (ctypes.c_int, [vp, vp, ctypes.c_int, vp, vp, vp, vp, vp, ctypes.c_uint32, vp]),
    "mhe_prng_apply_fixes": (ctypes.c_int, [vp, vp, ctypes.c_uint32, vp, vp]),
    "mhe_prng_small": (ctypes.c_int, [vp, vp, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, vp, vp, vp]),
}


class MheError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{msg} (code {code})")
        self.code = code


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        # One HIP runtime per process: PyTorch ships its own libamdhip64.so.7.  Importing torch
        # first makes libmhe.so's libamdhip64.so.7 dependency resolve to that same copy (same
        # SONAME); loading /opt/rocm's first and torch's second puts two runtimes in the process
        # and device initialisation fails.
        import torch  # noqa: F401

        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            # an A/B build from an older tree (MHE_LIB_PATH) may lack the newest entry points; the
            # in-tree library must export all of them (tests/test_capi.py)
            if LIB_PATH != _DEFAULT_LIB and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise MheError(rc, lib().mhe_last_error().decode())


def coeff_modulus_create(n, bit_sizes):
    """CoeffModulus::Create (modulus.cpp:143-185) -- host-only, no GPU needed."""
    bs = (ctypes.c_int * len(bit_sizes))(*bit_sizes)
    out = (ctypes.c_uint64 * len(bit_sizes))()
    _check(lib().mhe_coeff_modulus_create(n, bs, len(bit_sizes), out))
    return list(out)


def galois_elt_from_step(log_n, step):
    return int(lib().mhe_galois_elt_from_step(log_n, step))


def _torch():
    import torch

    return torch


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


class Engine:
    """One mhe_ctx: the key-level modulus chain on one device."""

    def __init__(self, log_n, moduli, device=0):
        torch = _torch()
        if not torch.cuda.is_available():
            raise RuntimeError("mhe.Engine needs a ROCm GPU (no CPU fallback)")
        self.log_n = log_n
        self.n = 1 << log_n
        self.moduli = [int(q) for q in moduli]
        self.K = len(self.moduli)
        self.device = device
        self.torch_device = torch.device("cuda", device)
        h = vp()
        arr = (ctypes.c_uint64 * self.K)(*self.moduli)
        _check(lib().mhe_ctx_create(ctypes.byref(h), log_n, arr, self.K, device))
        self._h = h

    def close(self):
        if getattr(self, "_enc", None):
            lib().mhe_encoder_destroy(self._enc)
            self._enc = None
        if getattr(self, "_h", None):
            lib().mhe_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ plumbing
    def stream(self):
        return ctypes.c_void_p(_torch().cuda.current_stream(self.torch_device).cuda_stream)

    def to_device(self, arr):
        torch = _torch()
        a = np.ascontiguousarray(arr, dtype=np.uint64)
        return torch.from_numpy(a.view(np.int64)).to(self.torch_device)

    def empty(self, *shape):
        torch = _torch()
        return torch.empty(*shape, dtype=torch.int64, device=self.torch_device)

    @staticmethod
    def to_host(t):
        return t.detach().cpu().numpy().view(np.uint64)

    def synchronize(self):
        _check(lib().mhe_stream_sync(self._h, self.stream()))

    def set_hoist(self, on, check=False):
        """mhe_ctx_set_hoist: hoisted rotations on / off for this context (check: every hoisted
        rotation is recomputed by the classic path and compared, mismatches counted)."""
        _check(lib().mhe_ctx_set_hoist(self._h, 1 if on else 0, 1 if check else 0))

    def hoist(self):
        """(effective hoisting on, check on) of this context."""
        on, chk = ctypes.c_int(), ctypes.c_int()
        _check(lib().mhe_ctx_get_hoist(self._h, ctypes.byref(on), ctypes.byref(chk)))
        return bool(on.value), bool(chk.value)

    def hoist_stats(self, reset=False):
        """(hoisted rotations, hoisted key-MAC launches, words that differed under check)."""
        r, m, b = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().mhe_hoist_stats(self._h, ctypes.byref(r), ctypes.byref(m), ctypes.byref(b), 1 if reset else 0))
        return r.value, m.value, b.value

    @staticmethod
    def alloc_stats(reset=False):
        """mhe_alloc_stats: (allocations that needed the cache released and a retry, failed ones), process-wide."""
        r, f = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().mhe_alloc_stats(ctypes.byref(r), ctypes.byref(f), 1 if reset else 0))
        return r.value, f.value

    def scratch_bytes(self):
        """mhe_scratch_bytes: (workspace, hoisting, Galois masks) device bytes and the stream count."""
        w, h, m, n = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
        _check(lib().mhe_scratch_bytes(self._h, ctypes.byref(w), ctypes.byref(h), ctypes.byref(m), ctypes.byref(n)))
        return w.value, h.value, m.value, n.value

    def reserve(self, max_limbs):
        _check(lib().mhe_ctx_reserve(self._h, max_limbs, self.stream()))

    @staticmethod
    def _pl(t):
        """(polys, limbs) of a [polys][limbs][n] or [limbs][n] tensor."""
        return (1, t.shape[0]) if t.dim() == 2 else (t.shape[0], t.shape[1])

    # ----------------------------------------------------------------- kernels
    SAMPLE_KINDS = {"ternary": 1, "cbd": 3}

    def prng_small(self, kind, limbs, seed, byte_offset=0, out=None, state=None):
        """[limbs][n] residues of sample_poly_ternary / sample_poly_cbd drawn from byte
        `byte_offset` of Blake2xbPRNG(seed) (mhe_prng_small; util/rlwe.cpp:21-38,101-133).
        `state` (int32 device tensor of 2): ternary writes the bytes its redraws used into
        state[0]; cbd given a state reads from byte_offset + state[0].  Returns (out, state)."""
        torch = _torch()
        out = self.empty(limbs, self.n) if out is None else out
        s = np.ascontiguousarray(np.array(seed, np.uint64))
        if state is None and kind == "ternary":
            state = torch.zeros(2, dtype=torch.int32, device=self.torch_device)
        _check(lib().mhe_prng_small(self._h, s.ctypes.data_as(ctypes.c_void_p), byte_offset, self.SAMPLE_KINDS[kind],
                                    limbs, _ptr(out), _ptr(state) if state is not None else None, self.stream()))
        return out, state

    def prng_uniform_bulk(self, limbs, seed, out=None, cap=1 << 16):
        """Bulk part of sample_poly_uniform over limbs 0..limbs-1 (mhe_prng_uniform_bulk): the reduced
        accepted words in out, and the (unordered) stream indices of the rejected words."""
        out = self.empty(limbs, self.n) if out is None else out
        s = np.ascontiguousarray(np.array(seed, np.uint64))
        idx = np.arange(limbs, dtype=np.int32)
        torch = _torch()
        rej = torch.zeros(cap, dtype=torch.int64, device=self.torch_device)
        cnt = torch.zeros(1, dtype=torch.int32, device=self.torch_device)
        _check(lib().mhe_prng_uniform_bulk(self._h, s.ctypes.data_as(ctypes.c_void_p), limbs,
                                           idx.ctypes.data_as(ctypes.c_void_p), idx.ctypes.data_as(ctypes.c_void_p),
                                           _ptr(out), _ptr(rej), _ptr(cnt), cap, self.stream()))
        c = int(cnt.item())
        return out, rej[:min(c, cap)].cpu().numpy().astype(np.uint64), c

    def ntt_forward(self, t, lazy=False):
        p, l = self._pl(t)
        _check(lib().mhe_ntt_forward(self._h, _ptr(t), p, l, int(lazy), self.stream()))
        return t

    def ntt_inverse(self, t, lazy=False):
        p, l = self._pl(t)
        _check(lib().mhe_ntt_inverse(self._h, _ptr(t), p, l, int(lazy), self.stream()))
        return t

    def add(self, a, b, out=None):
        out = self.empty(*a.shape) if out is None else out
        p, l = self._pl(a)
        _check(lib().mhe_add(self._h, _ptr(a), _ptr(b), _ptr(out), p, l, self.stream()))
        return out

    def sub(self, a, b, out=None):
        out = self.empty(*a.shape) if out is None else out
        p, l = self._pl(a)
        _check(lib().mhe_sub(self._h, _ptr(a), _ptr(b), _ptr(out), p, l, self.stream()))
        return out

    def negate(self, a, out=None):
        out = self.empty(*a.shape) if out is None else out
        p, l = self._pl(a)
        _check(lib().mhe_negate(self._h, _ptr(a), _ptr(out), p, l, self.stream()))
        return out

    def multiply_plain(self, a, pt, out=None):
        out = self.empty(*a.shape) if out is None else out
        p, l = self._pl(a)
        _check(lib().mhe_multiply_plain(self._h, _ptr(a), _ptr(pt), _ptr(out), p, l, self.stream()))
        return out

    def multiply_plain_sum(self, cts, pts, out=None, accumulate=False):
        """mhe_multiply_plain_sum: out (+)= sum_k cts[k] * pts[k] in one pass per 16 terms."""
        out = self.empty(*cts[0].shape) if out is None else out
        p, l = self._pl(cts[0])
        _check(lib().mhe_multiply_plain_sum(self._h, len(cts), self._ptrs(cts), self._ptrs(pts), _ptr(out),
                                            1 if accumulate else 0, p, l, self.stream()))
        return out

    def _scalar(self, fn, a, scalars, out):
        out = self.empty(*a.shape) if out is None else out
        p, l = self._pl(a)
        s = (ctypes.c_uint64 * l)(*[int(x) for x in scalars])
        _check(fn(self._h, _ptr(a), s, _ptr(out), p, l, self.stream()))
        return out

    def multiply_scalar(self, a, scalars, out=None):
        return self._scalar(lib().mhe_multiply_scalar, a, scalars, out)

    def add_scalar(self, a, scalars, out=None):
        return self._scalar(lib().mhe_add_scalar, a, scalars, out)

    def multiply(self, a, b, out3=None):
        L = a.shape[1]
        out3 = self.empty(3, L, self.n) if out3 is None else out3
        _check(lib().mhe_ct_multiply(self._h, _ptr(a), _ptr(b), _ptr(out3), L, self.stream()))
        return out3

    def square(self, a, out3=None):
        L = a.shape[1]
        out3 = self.empty(3, L, self.n) if out3 is None else out3
        _check(lib().mhe_ct_square(self._h, _ptr(a), _ptr(out3), L, self.stream()))
        return out3

    @staticmethod
    def _key_limbs(key):
        return key.shape[2]  # [digits][2][key_limbs][n]

    def key_prepare(self, key, fmt=None):
        """mhe_key_prepare(_as): convert `key` [digits][2][key_limbs][n] in place to one of the engine's
        key formats (fmt 1: residues of primes below 2^51 as doubles, 2: 48-bit planes for primes below
        2^48; None: mhe_key_prepare's default); switches given it stay bit-identical."""
        if fmt is None:
            _check(lib().mhe_key_prepare(self._h, _ptr(key), key.shape[0], self._key_limbs(key), self.stream()))
        else:
            _check(lib().mhe_key_prepare_as(self._h, _ptr(key), key.shape[0], self._key_limbs(key), int(fmt),
                                            self.stream()))
        return key

    def key_unprepare(self, key):
        """mhe_key_unprepare: back to SEAL's key layout."""
        _check(lib().mhe_key_unprepare(self._h, _ptr(key), key.shape[0], self._key_limbs(key), self.stream()))
        return key

    def key_is_prepared(self, key):
        return self.key_format(key) != 0

    def key_format(self, key):
        """0: SEAL's layout; 1: doubles; 2: 48-bit planes (mhe_key_is_prepared)."""
        v = ctypes.c_int()
        _check(lib().mhe_key_is_prepared(self._h, _ptr(key), self._key_limbs(key), ctypes.byref(v), self.stream()))
        return v.value

    def switch_key(self, ct, target, key):
        _check(lib().mhe_switch_key(self._h, _ptr(ct), _ptr(target), _ptr(key), self._key_limbs(key), ct.shape[1],
                                    self.stream()))
        return ct

    def relinearize(self, ct3, key):
        _check(lib().mhe_relinearize(self._h, _ptr(ct3), _ptr(key), self._key_limbs(key), ct3.shape[1],
                                     self.stream()))
        return ct3[:2]

    def apply_galois(self, ct, elt, key):
        _check(lib().mhe_apply_galois(self._h, _ptr(ct), elt, _ptr(key), self._key_limbs(key), ct.shape[1],
                                      self.stream()))
        return ct

    def apply_galois_to(self, ct, elt, key, out=None):
        out = self.empty(*ct.shape) if out is None else out
        _check(lib().mhe_apply_galois_to(self._h, _ptr(ct), _ptr(out), elt, _ptr(key), self._key_limbs(key),
                                         ct.shape[1], self.stream()))
        return out

    @staticmethod
    def _ptrs(ts):
        return (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])

    def apply_galois_batch(self, cts, elts, keys, outs=None):
        """mhe_apply_galois_batch: one batched launch sequence for len(cts) independent rotations."""
        outs = [self.empty(*c.shape) for c in cts] if outs is None else outs
        cnt = len(cts)
        e = (ctypes.c_uint32 * cnt)(*[int(x) for x in elts])
        kl = (ctypes.c_int * cnt)(*[self._key_limbs(k) for k in keys])
        _check(lib().mhe_apply_galois_batch(self._h, cnt, self._ptrs(cts), self._ptrs(outs), e, self._ptrs(keys), kl,
                                            cts[0].shape[1], self.stream()))
        return outs

    def rescale_batch(self, cts, outs=None):
        size, L = cts[0].shape[0], cts[0].shape[1]
        outs = [self.empty(size, L - 1, self.n) for _ in cts] if outs is None else outs
        _check(lib().mhe_rescale_batch(self._h, len(cts), self._ptrs(cts), self._ptrs(outs), size, L, self.stream()))
        return outs

    def switch_key_batch(self, cts, targets, keys):
        cnt = len(cts)
        kl = (ctypes.c_int * cnt)(*[self._key_limbs(k) for k in keys])
        _check(lib().mhe_switch_key_batch(self._h, cnt, self._ptrs(cts), self._ptrs(targets), self._ptrs(keys), kl,
                                          cts[0].shape[1], self.stream()))
        return cts

    def permute_galois(self, a, elt, out=None):
        out = self.empty(*a.shape) if out is None else out
        p, l = self._pl(a)
        _check(lib().mhe_permute_galois(self._h, _ptr(a), elt, _ptr(out), p, l, self.stream()))
        return out

    def rescale_to_next(self, ct, out=None):
        size, L = ct.shape[0], ct.shape[1]
        out = self.empty(size, L - 1, self.n) if out is None else out
        _check(lib().mhe_rescale_to_next(self._h, _ptr(ct), _ptr(out), size, L, self.stream()))
        return out

    def mod_switch_drop(self, ct, out=None):
        size, L = ct.shape[0], ct.shape[1]
        out = self.empty(size, L - 1, self.n) if out is None else out
        _check(lib().mhe_mod_switch_drop(self._h, _ptr(ct), _ptr(out), size, L, self.stream()))
        return out

    def modraise(self, ct1, L, out=None):
        """Bootstrapper::modraise_inplace lift: ct1 [size][1][n] coefficient form -> [size][L][n]."""
        size = ct1.shape[0]
        out = self.empty(size, L, self.n) if out is None else out
        _check(lib().mhe_modraise(self._h, _ptr(ct1), _ptr(out), size, L, self.stream()))
        return out

    def hmult(self, a, b, key, out=None):
        L = a.shape[1]
        out = self.empty(2, L - 1, self.n) if out is None else out
        _check(lib().mhe_hmult(self._h, _ptr(a), _ptr(b), _ptr(key), self._key_limbs(key), _ptr(out), L,
                               self.stream()))
        return out

    def hmult_batch(self, a_list, b_list, key, outs=None):
        """mhe_hmult_batch: len(a_list) independent HMults sharing the relinearization key."""
        L = a_list[0].shape[1]
        outs = [self.empty(2, L - 1, self.n) for _ in a_list] if outs is None else outs
        _check(lib().mhe_hmult_batch(self._h, len(a_list), self._ptrs(a_list), self._ptrs(b_list), _ptr(key),
                                     self._key_limbs(key), self._ptrs(outs), L, self.stream()))
        return outs

    def hmult_batch_raw(self, count, a_ptrs, b_ptrs, key_ptr, key_limbs, out_ptrs, L, stream):
        """Pointer-level batched HMult for the benchmark loop (ctypes pointer arrays)."""
        return lib().mhe_hmult_batch(self._h, count, a_ptrs, b_ptrs, key_ptr, key_limbs, out_ptrs, L, stream)

    def encode(self, values, scale, limbs, out=None, bound_limbs=None):
        """CKKSEncoder::encode -> NTT-form plaintext [limbs][n] on the device.  `bound_limbs`
        (default `limbs`) is the level SEAL's size checks use (encode at the first level then
        mod_switch_to, evaluator.cpp:287-310)."""
        self._encoder()
        v = np.asarray(values)
        re = np.ascontiguousarray(v.real, np.float64)
        im = np.ascontiguousarray(v.imag, np.float64) if np.iscomplexobj(v) else None
        out = self.empty(limbs, self.n) if out is None else out
        dp = ctypes.POINTER(ctypes.c_double)
        _check(lib().mhe_ckks_encode_at(self._h, self._enc, re.ctypes.data_as(dp),
                                        im.ctypes.data_as(dp) if im is not None else None, re.size, scale,
                                        limbs if bound_limbs is None else bound_limbs, limbs, _ptr(out),
                                        self.stream()))
        return out

    def _encoder(self):
        if getattr(self, "_enc", None) is None:
            h = vp()
            _check(lib().mhe_encoder_create(ctypes.byref(h), self.log_n))
            self._enc = h
        return self._enc

    def decode(self, plain, scale, sparse_slots=0):
        """CKKSEncoder::decode: device NTT-form plaintext [limbs][n] -> complex numpy slots."""
        limbs = plain.shape[-2]
        cnt = sparse_slots or self.n // 2
        re = np.zeros(cnt, np.float64)
        im = np.zeros(cnt, np.float64)
        dp = ctypes.POINTER(ctypes.c_double)
        _check(lib().mhe_ckks_decode(self._h, self._encoder(), _ptr(plain), limbs, scale, sparse_slots,
                                     re.ctypes.data_as(dp), im.ctypes.data_as(dp), self.stream()))
        return re + 1j * im

    def encode_scalar(self, value, scale, limbs, bound_limbs=None):
        out = (ctypes.c_uint64 * limbs)()
        _check(lib().mhe_ckks_encode_scalar_at(self._h, value, scale, limbs if bound_limbs is None else bound_limbs,
                                               limbs, out))
        return list(out)

    def hmult_raw(self, a_ptr, b_ptr, key_ptr, key_limbs, out_ptr, L, stream):
        """Pointer-level HMult for the benchmark loop (no tensor bookkeeping)."""
        return lib().mhe_hmult(self._h, a_ptr, b_ptr, key_ptr, key_limbs, out_ptr, L, stream)
