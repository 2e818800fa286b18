"""SEAL's randomness in the oracle (oracle/seal_random.c), pinned independently.

* BLAKE2b/BLAKE2Xb: hashlib.blake2b pins a pure-Python BLAKE2b below on standard parameter blocks
  (keyed, fanout/depth/leaf/node_offset/inner variations); hashlib refuses depth 0, which the
  BLAKE2Xb output nodes use (util/blake2xb.c:111-133), so those are checked through the pinned
  pure-Python compression.
* Blake2xbPRNG (randomgen.cpp:160-195): 4096-byte buffers, buffer c = BLAKE2Xb(4096, counter c,
  64-byte seed).
* samplers (util/rlwe.cpp:21-162) restated in plain Python from the pinned stream and compared with
  the C restatement, including libstdc++'s Lemire downscaling for uniform_int_distribution.
No GPU: these are the -m "not gpu" pins of the oracle; GPU parity is in test_gpu_random.py.
"""
import hashlib
import os
import struct
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

M64 = (1 << 64) - 1
IV = [0x6A09E667F3BCC908, 0xBB67AE8584CAA73B, 0x3C6EF372FE94F82B, 0xA54FF53A5F1D36F1,
      0x510E527FADE682D1, 0x9B05688C2B3E6C1F, 0x1F83D9ABFB41BD6B, 0x5BE0CD19137E2179]
SIGMA = [
    [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15],
    [14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3],
    [11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4],
    [7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8],
    [9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13],
    [2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9],
    [12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11],
    [13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10],
    [6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5],
    [10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0],
]


def _rotr(x, r):
    return ((x >> r) | (x << (64 - r))) & M64


def _compress(h, block, t, last):
    m = struct.unpack("<16Q", block)
    v = list(h) + list(IV)
    v[12] ^= t & M64
    v[13] ^= t >> 64
    if last:
        v[14] ^= M64

    def g(a, b, c, d, x, y):
        v[a] = (v[a] + v[b] + x) & M64
        v[d] = _rotr(v[d] ^ v[a], 32)
        v[c] = (v[c] + v[d]) & M64
        v[b] = _rotr(v[b] ^ v[c], 24)
        v[a] = (v[a] + v[b] + y) & M64
        v[d] = _rotr(v[d] ^ v[a], 16)
        v[c] = (v[c] + v[d]) & M64
        v[b] = _rotr(v[b] ^ v[c], 63)

    for r in range(12):
        s = SIGMA[r % 10]
        g(0, 4, 8, 12, m[s[0]], m[s[1]])
        g(1, 5, 9, 13, m[s[2]], m[s[3]])
        g(2, 6, 10, 14, m[s[4]], m[s[5]])
        g(3, 7, 11, 15, m[s[6]], m[s[7]])
        g(0, 5, 10, 15, m[s[8]], m[s[9]])
        g(1, 6, 11, 12, m[s[10]], m[s[11]])
        g(2, 7, 8, 13, m[s[12]], m[s[13]])
        g(3, 4, 9, 14, m[s[14]], m[s[15]])
    return [h[i] ^ v[i] ^ v[i + 8] for i in range(8)]


def py_blake2b(data, digest_size=64, key=b"", fanout=1, depth=1, leaf_size=0, node_offset=0, node_depth=0,
               inner_size=0):
    """BLAKE2b with an explicit parameter block (RFC 7693 + the tree parameters)."""
    param = bytes([digest_size, len(key), fanout, depth]) + struct.pack("<I", leaf_size) + \
        struct.pack("<Q", node_offset) + bytes([node_depth, inner_size]) + bytes(46)
    h = [IV[i] ^ struct.unpack_from("<Q", param, 8 * i)[0] for i in range(8)]
    msg = (key + bytes(128 - len(key)) if key else b"") + bytes(data)
    t = 0
    if not msg:
        return b"".join(struct.pack("<Q", x) for x in _compress(h, bytes(128), 0, True))[:digest_size]
    blocks = [msg[i:i + 128] for i in range(0, len(msg), 128)]
    for i, blk in enumerate(blocks):
        last = i == len(blocks) - 1
        t += len(blk)
        h = _compress(h, blk + bytes(128 - len(blk)), t, last)
    return b"".join(struct.pack("<Q", x) for x in h)[:digest_size]


def py_blake2xb(outlen, data, key):
    """BLAKE2Xb (util/blake2xb.c): root with xof_length in the upper node_offset word, then output
    node i = BLAKE2b(root) with {fanout 0, depth 0, leaf 64, node_offset i, inner 64}."""
    root = py_blake2b(data, 64, key, 1, 1, 0, outlen << 32, 0, 0)
    out = b""
    i = 0
    while len(out) < outlen:
        bs = min(64, outlen - len(out))
        out += py_blake2b(root, bs, b"", 0, 0, 64, i | (outlen << 32), 0, 64)
        i += 1
    return out


@pytest.mark.parametrize("kw", [
    dict(),
    dict(key=bytes(range(64))),
    dict(key=b"k" * 17, digest_size=32),
    dict(fanout=3, depth=2, leaf_size=64, node_offset=(4096 << 32) | 7, node_depth=1, inner_size=64),
    dict(key=bytes(range(64)), node_offset=4096 << 32),
])
@pytest.mark.parametrize("size", [0, 8, 127, 128, 129, 300])
def test_py_blake2b_matches_hashlib(kw, size):
    data = bytes((7 * i + 3) & 0xFF for i in range(size))
    ds = kw.get("digest_size", 64)
    want = hashlib.blake2b(data, **{k: v for k, v in kw.items() if k not in ("node_offset",)},
                           node_offset=kw.get("node_offset", 0)).digest()
    got = py_blake2b(data, ds, kw.get("key", b""), kw.get("fanout", 1), kw.get("depth", 1), kw.get("leaf_size", 0),
                     kw.get("node_offset", 0), kw.get("node_depth", 0), kw.get("inner_size", 0))
    assert got == want


@pytest.mark.parametrize("outlen", [1, 63, 64, 65, 200, 4096])
def test_oracle_blake2xb(outlen):
    key = bytes(range(64))
    msg = struct.pack("<Q", 3)
    # the root node through hashlib itself (depth 1 is representable)
    root = hashlib.blake2b(msg, digest_size=64, key=key, fanout=1, depth=1, node_offset=outlen << 32).digest()
    assert root == py_blake2b(msg, 64, key, 1, 1, 0, outlen << 32)
    assert O.blake2xb(outlen, msg, key) == py_blake2xb(outlen, msg, key)


SEED = [1, 2, 3, 4, 5, 6, 7, 8]  # SEAL's documented debug seed (randomgen.h / tests/seal/randomgen.cpp:108)


def py_stream(seed, count):
    key = b"".join(struct.pack("<Q", w) for w in seed)
    out = b""
    c = 0
    while len(out) < count:
        out += py_blake2xb(4096, struct.pack("<Q", c), key)
        c += 1
    return out[:count]


def test_prng_stream():
    assert O.prng_bytes(SEED, 4096 + 200) == py_stream(SEED, 4096 + 200)


class _Stream:
    def __init__(self, seed):
        self.b = py_stream(seed, 3 * 4096 * 16)
        self.p = 0

    def take(self, k):
        r = self.b[self.p:self.p + k]
        self.p += k
        return r

    def u32(self):
        return struct.unpack("<I", self.take(4))[0]

    def uniform_int(self, a, b):
        # libstdc++ 11 uniform_int_distribution<u64> over a 32-bit URBG (Lemire)
        er = b - a + 1
        prod = self.u32() * er
        low = prod & 0xFFFFFFFF
        if low < er:
            thr = ((1 << 32) - er) % er
            while low < thr:
                prod = self.u32() * er
                low = prod & 0xFFFFFFFF
        return (prod >> 32) + a


def test_samplers_match_plain_restatement():
    log_n = 6
    n = 1 << log_n
    moduli = O.coeff_modulus_create(n, [30, 30, 30])
    oc = O.Context(log_n, moduli)
    qs = [int(q) for q in moduli]

    # ternary
    st = _Stream(SEED)
    v = [st.uniform_int(0, 2) - 1 for _ in range(n)]
    want = np.array([[x % q for x in v] for q in qs], np.uint64)
    assert np.array_equal(oc.sample(SEED, "ternary", 3), want)
    # cbd
    st = _Stream(SEED)
    cbd = []
    for _ in range(n):
        x = bytearray(st.take(6))
        x[2] &= 0x1F
        x[5] &= 0x1F
        cbd.append(sum(bin(b).count("1") for b in x[:3]) - sum(bin(b).count("1") for b in x[3:]))
    want = np.array([[x % q for x in cbd] for q in qs], np.uint64)
    assert np.array_equal(oc.sample(SEED, "cbd", 3), want)
    # uniform: bulk, then in-order redraws (rlwe.cpp:146-160)
    st = _Stream(SEED)
    bulk = list(struct.unpack(f"<{3 * n}Q", st.take(3 * n * 8)))
    out = []
    for j, q in enumerate(qs):
        mm = M64 - (M64 % q) - 1
        for i in range(n):
            r = bulk[j * n + i]
            while r >= mm:
                r = struct.unpack("<Q", st.take(8))[0]
            out.append(r % q)
    assert np.array_equal(oc.sample(SEED, "uniform", 3), np.array(out, np.uint64).reshape(3, n))
    # sparse ternary (hw 5): SEAL's inclusive position range (index n can be drawn), with a draw
    # of n redrawn (SEAL would write a non-residue into limb 1's coefficient 0)
    st = _Stream(SEED)
    arr = [0] * (3 * n)
    w = 0
    while w < 5:
        idx = st.uniform_int(0, n)
        if idx >= n or arr[idx] != 0:
            continue
        r = 2 * st.uniform_int(0, 1)
        for j, q in enumerate(qs):
            arr[idx + j * n] = q - 1 if r == 0 else r - 1
        w += 1
    assert np.array_equal(oc.sample(SEED, "sparse_ternary", 3, hw=5), np.array(arr, np.uint64).reshape(3, n))


def test_sparse_ternary_redraws_position_n():
    """SEAL's sparse sampler draws positions from [0, n] inclusive; a draw of n would write limb 1's
    coefficient 0 with limb 0's residue (not a ring element).  For a seed whose draws hit n, the
    oracle (like the engine, seal/random.cpp) redraws it: the key has exactly hw nonzero positions,
    each the same +-1 in every limb."""
    log_n = 6
    n = 1 << log_n
    moduli = O.coeff_modulus_create(n, [30, 40, 30])
    oc = O.Context(log_n, moduli)
    qs = [int(q) for q in moduli]
    hw = 32
    hit = None
    for s0 in range(1, 400):
        seed = [s0, 2, 3, 4, 5, 6, 7, 8]
        st = _Stream(seed)
        taken, w = set(), 0
        drew_n = False
        while w < hw:
            idx = st.uniform_int(0, n)
            if idx == n:
                drew_n = True
            if idx >= n or idx in taken:
                continue
            st.uniform_int(0, 1)
            taken.add(idx)
            w += 1
        if drew_n:
            hit = seed
            break
    assert hit is not None
    key = oc.sample(hit, "sparse_ternary", 3, hw=hw).astype(object)
    nz = [i for i in range(n) if key[0][i] != 0]
    assert len(nz) == hw
    for i in range(n):
        vals = {(int(key[j][i]) + 1) % qs[j] - 1 for j in range(3)}  # residues -> {-1, 0, 1}
        assert len(vals) == 1 and vals <= {-1, 0, 1}


def test_uniform_rejection_path_exercised():
    """A 61-bit modulus rejects about 2^64 mod q / 2^64 of the words; over 4 x 64 words some are
    redrawn, so the in-order redraw path of sample_poly_uniform runs."""
    log_n = 6
    n = 1 << log_n
    q = 3 << 59  # an NTT prime near 1.5 * 2^60: 2^64 mod q ~ 0.67 q, about 1 word in 16 redrawn
    q += 1
    while not O.is_prime(q):
        q += 2 * n
    oc = O.Context(log_n, [q])
    mm = M64 - (M64 % q) - 1
    redraws = 0
    for s0 in range(1, 5):
        seed = [s0] + SEED[1:]
        st = _Stream(seed)
        bulk = list(struct.unpack(f"<{n}Q", st.take(n * 8)))
        out = []
        for r in bulk:
            while r >= mm:
                redraws += 1
                r = struct.unpack("<Q", st.take(8))[0]
            out.append(r % q)
        assert np.array_equal(oc.sample(seed, "uniform", 1)[0], np.array(out, np.uint64))
    assert redraws > 0
