"""Device samplers of key generation and encryption (csrc/sample.hip) against the oracle's
sequential restatement of SEAL's samplers on Blake2xbPRNG (oracle/seal_random.c, pinned by hashlib
in test_seal_random.py): sample_poly_ternary / sample_poly_cbd at stream offsets, and the bulk of
sample_poly_uniform with its rejected indices redrawn in order from the stream tail
(util/rlwe.cpp:21-162)."""
import struct

import numpy as np
import pytest

import mhe
import oracle as O

SEED = [1, 2, 3, 4, 5, 6, 7, 8]
M64 = (1 << 64) - 1


def _heavy_reject_primes(log_n, count):
    """NTT primes just above 1.5 * 2^60: 2^64 mod q ~ 0.67 q, so ~1 word in 16 is redrawn."""
    out, q = [], (3 << 59) + 1
    while len(out) < count:
        if O.is_prime(q):
            out.append(q)
        q += 2 << log_n
    return out


def _eng(log_n, bits):
    moduli = mhe.coeff_modulus_create(1 << log_n, bits) if bits else _heavy_reject_primes(log_n, 4)
    return mhe.Engine(log_n, moduli, device=0), O.Context(log_n, moduli), moduli


def _small_from_stream(kind, raw, n, moduli, limbs):
    if kind == "ternary":
        w = np.frombuffer(raw[:4 * n], dtype=np.uint32).astype(np.uint64)
        v = ((w * np.uint64(3)) >> np.uint64(32)).astype(np.int64) - 1
    else:
        b = np.frombuffer(raw[:6 * n], dtype=np.uint8).reshape(n, 6).copy()
        b[:, 2] &= 0x1F
        b[:, 5] &= 0x1F
        pc = np.unpackbits(b, axis=1).reshape(n, 6, 8).sum(axis=2).astype(np.int64)
        v = pc[:, 0] + pc[:, 1] + pc[:, 2] - pc[:, 3] - pc[:, 4] - pc[:, 5]
    return np.stack([np.where(v >= 0, v, v + int(q)).astype(np.uint64) for q in moduli[:limbs]])


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["ternary", "cbd"])
@pytest.mark.parametrize("offset", [0, 64, 4 * 4096, 10 * 4096 + 128])
def test_small_samplers(kind, offset):
    log_n = 12
    eng, oc, moduli = _eng(log_n, [50, 40, 40, 50])
    n = 1 << log_n
    got, state = eng.prng_small(kind, 3, SEED, offset)
    if state is not None:
        assert state.cpu().tolist() == [0, 0]  # no zero word: no redraw
    got = mhe.Engine.to_host(got)
    raw = O.prng_bytes(SEED, offset + 6 * n)[offset:]
    assert np.array_equal(got, _small_from_stream(kind, raw, n, moduli, 3))
    if offset == 0:
        assert np.array_equal(got, oc.sample(SEED, kind, 3))


@pytest.mark.gpu
@pytest.mark.parametrize("log_n,bits", [(12, None), (14, [51] + [46] * 6 + [51])])
def test_uniform_bulk_and_redraws(log_n, bits):
    eng, oc, moduli = _eng(log_n, bits)
    n, limbs = 1 << log_n, len(moduli)
    out, rej, count = eng.prng_uniform_bulk(limbs, SEED)
    got = mhe.Engine.to_host(out).copy()
    raw = np.frombuffer(O.prng_bytes(SEED, limbs * n * 8 + 64 * 4096), dtype=np.uint64)
    bulk = raw[:limbs * n]
    mm = np.array([M64 - (M64 % int(q)) - 1 for q in moduli], dtype=np.uint64)
    want_rej = np.nonzero(bulk >= np.repeat(mm, n))[0].astype(np.uint64)
    assert count == len(want_rej) and np.array_equal(np.sort(rej), want_rej)
    # in-order redraws from the words after the bulk (what seal::rnd::sample_uniform_dev does)
    t = limbs * n
    for g in np.sort(rej):
        l = int(g) // n
        while raw[t] >= mm[l]:
            t += 1
        got[l, int(g) % n] = int(raw[t]) % int(moduli[l])
        t += 1
    assert np.array_equal(got, oc.sample(SEED, "uniform", limbs))
    if bits is None:
        assert count > 100  # the redraw path is exercised


@pytest.mark.gpu
def test_cbd_after_shifted_ternary():
    """CBD reads from byte_offset + state[0]: the offset a ternary redraw leaves behind (4-byte
    aligned, not 64) -- the 3-4 block path of k_prng_cbd."""
    log_n = 12
    eng, oc, moduli = _eng(log_n, [50, 40, 40, 50])
    n = 1 << log_n
    torch = pytest.importorskip("torch")
    for extra in (4, 60, 68):
        state = torch.tensor([extra, 0], dtype=torch.int32, device=eng.torch_device)
        got, _ = eng.prng_small("cbd", 2, SEED, 4 * n, state=state)
        raw = O.prng_bytes(SEED, 4 * n + extra + 6 * n)[4 * n + extra:]
        assert np.array_equal(mhe.Engine.to_host(got), _small_from_stream("cbd", raw, n, moduli, 2))


@pytest.mark.gpu
def test_ternary_redraw_path():
    """A seed whose ternary draws hit a zero word (tests/golden/ternary_redraw_seed.json, found by
    find_ternary_redraw_seed.c): the redraw moves every later draw; the GPU's sequential fix and the
    CBD offsets after it follow SEAL's stream (oracle sample_poly_ternary / cbd on one PRNG)."""
    import json
    import os

    fx = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ternary_redraw_seed.json")))
    seed = [fx["seed0"], 2, 3, 4, 5, 6, 7, 8]
    log_n = fx["log_n"]
    eng, oc, moduli = _eng(log_n, [50, 40, 40, 50])
    n = 1 << log_n
    u, state = eng.prng_small("ternary", 3, seed, 0)
    assert np.array_equal(mhe.Engine.to_host(u), oc.sample(seed, "ternary", 3))
    extra = int(state[0].item())
    assert extra >= 4 and extra % 4 == 0
    e0, _ = eng.prng_small("cbd", 3, seed, 4 * n, state=state)
    raw = O.prng_bytes(seed, 4 * n + extra + 6 * n)[4 * n + extra:]
    assert np.array_equal(mhe.Engine.to_host(e0), _small_from_stream("cbd", raw, n, moduli, 3))
