"""TEST INFRASTRUCTURE (oracle): a CPU restatement of the modified SEAL 3.6.6 Evaluator's
scale-aware operations over the oracle's exact primitives (mhe_oracle.c via oracle.py).  Only
tests/ use it, as the checker; nothing in the product path imports it.

Paths are relative to cnn_ckks/cpu-ckks/single-key/seal-modified-3.6.6/native/src/seal/.

A ciphertext is OCt(data [size][L][n] u64, scale); L = the number of data primes of its level,
the first level having `first` primes (SEALContext::first_context_data).  Every operation follows
the reference's C++ line by line, including the double-precision scale bookkeeping and the
"scale out of bounds" checks, so a ciphertext's words AND its scale can be compared with the GPU
surface's bit for bit.
"""
import math

import numpy as np

import oracle as O


class OCt:
    __slots__ = ("data", "scale")

    def __init__(self, data, scale):
        self.data = np.ascontiguousarray(data, np.uint64)
        self.scale = float(scale)

    @property
    def L(self):
        return self.data.shape[1]

    @property
    def size(self):
        return self.data.shape[0]

    def copy(self):
        return OCt(self.data.copy(), self.scale)


def are_close(a, b):
    """util::are_close<double> (util/common.h): |a - b| < epsilon * max(|a|, |b|, 1)."""
    return abs(a - b) < np.finfo(np.float64).eps * max(abs(a), abs(b), 1.0)


class Evaluator:
    def __init__(self, ctx, first, relin_key=None, galois_keys=None):
        """ctx: oracle Context over the key-level chain; first: data primes of the first level;
        relin_key: [digits][2][K][n]; galois_keys: {galois_elt: key [digits][2][K][n]}."""
        self.ctx = ctx
        self.first = first
        self.relin_key = relin_key
        self.galois_keys = galois_keys or {}

    # ------------------------------------------------------------------ helpers
    def _bits(self, L):
        return self.ctx.total_bits(L)

    def _check_scale(self, scale, L):
        """is_scale_within_bounds (evaluator.cpp:29-47) for the level with L primes."""
        if scale <= 0 or int(math.log2(scale)) >= self._bits(L):
            raise ValueError("scale out of bounds")

    # ------------------------------------------------------------------ SEAL 3.6 ops
    def add_inplace(self, a, b):
        """evaluator.cpp:103-164 (CKKS, equal sizes)."""
        if a.L != b.L:
            raise ValueError("encrypted1 and encrypted2 parameter mismatch")
        if not are_close(a.scale, b.scale):
            raise ValueError("scale mismatch")
        a.data = self.ctx.add(a.data, b.data)

    def sub_inplace(self, a, b):
        """evaluator.cpp:166-246."""
        if a.L != b.L:
            raise ValueError("encrypted1 and encrypted2 parameter mismatch")
        if not are_close(a.scale, b.scale):
            raise ValueError("scale mismatch")
        a.data = self.ctx.sub(a.data, b.data)

    def multiply_inplace(self, a, b):
        """ckks_multiply (evaluator.cpp:673-814): tensor product, scale = s1 * s2."""
        if a.L != b.L:
            raise ValueError("encrypted1 and encrypted2 parameter mismatch")
        new_scale = a.scale * b.scale
        self._check_scale(new_scale, a.L)
        a.data = self.ctx.square(a.data) if a is b else self.ctx.multiply(a.data, b.data)
        a.scale = new_scale

    def relinearize_inplace(self, a):
        """relinearize_internal (evaluator.cpp:1061-1116)."""
        if a.size == 3:
            a.data = self.ctx.relinearize(a.data, self.relin_key)

    def rescale_to_next_inplace(self, a):
        """mod_switch_scale_to_next (evaluator.cpp:1118-1181): divide_and_round_q_last_ntt, scale /= q_last."""
        if a.L < 2:
            raise ValueError("end of modulus switching chain reached")
        q_last = float(self.ctx.moduli[a.L - 1])
        new_scale = a.scale / q_last
        self._check_scale(new_scale, a.L - 1)
        a.data = self.ctx.rescale(a.data)
        a.scale = new_scale

    def mod_switch_to_inplace(self, a, L):
        """mod_switch_drop_to_next repeated (evaluator.cpp:1183-1246, 1283-1376)."""
        if L > a.L:
            raise ValueError("cannot switch to higher level modulus")
        while a.L > L:
            self._check_scale(a.scale, a.L - 1)
            a.data = np.ascontiguousarray(a.data[:, : a.L - 1])

    def multiply_plain_inplace(self, a, pt, pt_scale):
        """multiply_plain_ntt (evaluator.cpp:1726-1761, 1891-1930): pt [L][n] NTT form."""
        new_scale = a.scale * pt_scale
        self._check_scale(new_scale, a.L)
        a.data = self.ctx.multiply_plain(a.data, pt)
        a.scale = new_scale

    def encode_const(self, value, scale, L):
        """CKKSEncoder::encode(double, scale) at the first level (ckks.cpp:78-200) then
        mod_switch_to_inplace(plain, parms_id) (evaluator.cpp:1248-1281): the residues of the
        first L primes, each broadcast over the n NTT coefficients."""
        r = self.ctx.encode_scalar(value, scale, self.first)[:L]
        return np.repeat(np.array(r, np.uint64)[:, None], self.ctx.n, axis=1)

    def multiply_const(self, a, value):
        """multiply_const (evaluator.cpp:294-301 + evaluator.h:1198-1204): encode(value,
        encrypted.scale()), mod switch, multiply_plain; the product's scale is scale^2."""
        out = a.copy()
        pt = self.encode_const(value, a.scale, a.L)
        self.multiply_plain_inplace(out, pt, a.scale)
        return out

    def add_const_inplace(self, a, value):
        """add_const_inplace (evaluator.cpp:287-292): add_plain of the constant at the ct's scale."""
        pt = self.encode_const(value, a.scale, a.L)
        a.data = a.data.copy()
        a.data[0] = self.ctx.add(a.data[0], pt)

    def multiply_vector_plain(self, a, values):
        """multiply_vector_inplace (evaluator.cpp:303-310): encode(values, encrypted.scale()) at the
        first level, mod switch, multiply_plain."""
        pt = self.ctx.encode(values, a.scale, self.first)[: a.L]
        out = a.copy()
        self.multiply_plain_inplace(out, np.ascontiguousarray(pt), a.scale)
        return out

    def rotate_vector(self, a, step):
        """rotate_internal (evaluator.cpp:2224-2279) for a step whose key is present."""
        elt = O.galois_elt_from_step(self.ctx.n, step)
        return OCt(self.ctx.apply_galois(a.data, elt, self.galois_keys[elt]), a.scale)

    # ------------------------------------------------ modified SEAL: *_reduced_error
    def _adjust(self, hi, lo):
        """The unequal-level branch shared by add/sub/multiply_inplace_reduced_error
        (evaluator.cpp:322-338 / 345-361 and the sub/mul copies): the higher ciphertext `hi` is
        multiplied by scale_adjust = lo.scale * q_top / hi.scale^2 (q_top = the last prime of hi's
        level), its scale forced to lo.scale * q_top, rescaled and mod-switched to lo's level."""
        q_top = float(self.ctx.moduli[hi.L - 1])
        scale_adjust = lo.scale * q_top / (hi.scale * hi.scale)
        adj = self.multiply_const(hi, scale_adjust)
        adj.scale = lo.scale * q_top
        self.rescale_to_next_inplace(adj)
        self.mod_switch_to_inplace(adj, lo.L)
        return adj

    def _reduced(self, a, b, op):
        if a.L == b.L:
            a.scale = b.scale
            op(a, b)
            return
        if a.L < b.L:
            # evaluator.cpp:322-338: b is adjusted down to a's level, a takes its scale
            adj = self._adjust(b, a)
            a.scale = adj.scale
            op(a, adj)
        else:
            # evaluator.cpp:340-361: a is adjusted down to b's level, then a = adj (op) b
            adj = self._adjust(a, b)
            adj.scale = b.scale
            op(adj, b)
            a.data, a.scale = adj.data, adj.scale

    def add_inplace_reduced_error(self, a, b):
        """evaluator.cpp:312-362."""
        self._reduced(a, b, self.add_inplace)

    def sub_inplace_reduced_error(self, a, b):
        """evaluator.cpp:364-416."""
        self._reduced(a, b, self.sub_inplace)

    def multiply_inplace_reduced_error(self, a, b):
        """evaluator.cpp:418-486: the same adjustment, multiply, then relinearize (both branches)."""
        self._reduced(a, b, self.multiply_inplace)
        self.relinearize_inplace(a)
