"""SEAL 3.6 serialization of the drop-in surface (fhe-gpt-2_amd/seal/serialize.cpp).

* parms_id is SEAL's: BLAKE2b-256 over the u64 words [scheme=2, n, coeff moduli..., 0]
  (SEAL/encryptionparams.cpp:124-158, SEAL/util/hash.h:30-37); checked here against Python's
  hashlib.blake2b, an independent implementation of RFC 7693 (no GPU).
* save/load round trips, decrypt-after-load and rejection of corrupt streams run on the GPU
  (tests/cpp/serialize_test.cpp, after the reference's CiphertextTest.SaveLoadCiphertext /
  PlaintextTest.SaveLoadPlaintext); the files it writes are then parsed here against the SEAL
  format (SEAL/serialization.h:60-120, ciphertext.cpp:183-230, plaintext.cpp:204-230,
  dynarray.h:652-680)."""
import hashlib
import os
import struct
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "fhe-gpt-2_amd")
EXE = os.path.join(ROOT, "build", "serialize_test")


def _build():
    subprocess.check_call(["make", "-s", "-C", os.path.join(PKG, "seal"), "all", "test"])


def seal_parms_id(n, moduli):
    words = [2, n] + list(moduli) + [0]
    d = hashlib.blake2b(struct.pack(f"<{len(words)}Q", *words), digest_size=32).digest()
    return list(struct.unpack("<4Q", d))


def test_blake2b_kat():
    # RFC 7693 Appendix A / the BLAKE2 reference test vector: BLAKE2b-512("abc"); hashlib is the
    # checker used for parms_id below, so pin it first
    assert hashlib.blake2b(b"abc").hexdigest().startswith("ba80a53f981c4d0d6a2797b69f12f6e9")


def test_parms_id_matches_seal_hash():
    _build()
    out = subprocess.check_output([EXE, "parms"], text=True)
    lines = out.strip().splitlines()
    assert len(lines) == 4
    for i in (0, 2):
        f = lines[i].split()
        n, moduli = int(f[1]), [int(x) for x in f[2:]]
        got = [int(x, 16) for x in lines[i + 1].split()[1:]]
        assert got == seal_parms_id(n, moduli), (n, got)


def _header(b, off=0):
    magic, hsize, vmaj, vmin, mode, res, size = struct.unpack_from("<HBBBBHQ", b, off)
    assert (magic, hsize, vmaj, vmin, mode, res) == (0xA15E, 16, 3, 6, 0, 0)
    return size


@pytest.mark.gpu
def test_save_load_roundtrip(tmp_path):
    _build()
    r = subprocess.run([EXE, "roundtrip", str(tmp_path)], capture_output=True, text=True, timeout=300)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    moduli = [int(x) for x in open(tmp_path / "moduli.txt").read().split()]
    n = 1 << 13
    first_id = [int(x, 16) for x in r.stdout.split("first_parms_id")[1].split("\n")[0].split()]
    assert first_id == seal_parms_id(n, moduli)
    # ciphertext: header | parms_id | ntt byte | size | n | L | scale | DynArray(header | count | data)
    b = open(tmp_path / "ct.bin", "rb").read()
    assert _header(b) == len(b)
    pid = list(struct.unpack_from("<4Q", b, 16))
    ntt, size, nn, L, scale = struct.unpack_from("<BQQQd", b, 48)
    assert pid == first_id and ntt == 1 and size == 2 and nn == n and L == len(moduli) and scale == 2.0**46
    off = 48 + 1 + 24 + 8
    assert _header(b, off) == len(b) - off
    (count,) = struct.unpack_from("<Q", b, off + 16)
    assert count == size * L * n
    data = np.frombuffer(b, dtype="<u8", count=count, offset=off + 24).reshape(size, L, n)
    assert (data < np.array(moduli, dtype=np.uint64)[None, :, None]).all()
    # plaintext: header | parms_id | coeff_count | scale | DynArray
    p = open(tmp_path / "pt.bin", "rb").read()
    assert _header(p) == len(p)
    assert list(struct.unpack_from("<4Q", p, 16)) == first_id
    cc, pscale = struct.unpack_from("<Qd", p, 48)
    assert cc == L * n and pscale == 2.0**46
    assert _header(p, 64) == len(p) - 64
    assert struct.unpack_from("<Q", p, 80)[0] == cc
    # relin keys: header | key parms_id | dim1 = 1 | dim2 = K - 1 | K - 1 PublicKeys (size 2, key level)
    k = open(tmp_path / "relin.bin", "rb").read()
    assert _header(k) == len(k)
    K = len(moduli) + 1
    key_id = list(struct.unpack_from("<4Q", k, 16))
    dim1, dim2 = struct.unpack_from("<QQ", k, 48)
    assert dim1 == 1 and dim2 == K - 1
    off = 64
    for _ in range(dim2):
        size = _header(k, off)
        assert list(struct.unpack_from("<4Q", k, off + 16)) == key_id
        ntt, sz, nn, kl = struct.unpack_from("<BQQQ", k, off + 48)
        assert (ntt, sz, nn, kl) == (1, 2, n, K)
        off += size
    assert off == len(k)


def _parse_ct(b, off=0):
    """One Ciphertext record at `off`: (end offset, fields, c0/c1 or c0 + seed)."""
    size = _header(b, off)
    ntt, sz, nn, L, scale = struct.unpack_from("<BQQQd", b, off + 48)
    d = off + 16 + 32 + 1 + 24 + 8
    dsize = _header(b, d)
    (count,) = struct.unpack_from("<Q", b, d + 16)
    data = np.frombuffer(b, dtype="<u8", count=count, offset=d + 24).reshape(-1, L, nn)
    seed = None
    if count == L * nn:  # seeded: UniformRandomGeneratorInfo follows the DynArray
        i = d + dsize
        assert _header(b, i) == 81
        assert b[i + 16] == 1  # prng_type::blake2xb
        seed = list(struct.unpack_from("<8Q", b, i + 17))
        assert i + 81 == off + size
    else:
        assert d + dsize == off + size
    return off + size, dict(ntt=ntt, size=sz, n=nn, L=L, scale=scale), data, seed


@pytest.mark.gpu
def test_seeded_save_expands_with_the_oracle_prng(tmp_path):
    """SEAL's seeded save (ciphertext.cpp:148-239): a Serializable ciphertext / relin key is written
    with c0 only plus a Blake2xb UniformRandomGeneratorInfo per encryption, and that seed expanded by
    the oracle's own restatement of sample_poly_uniform (oracle/seal_random.c, rlwe.cpp:133-162)
    gives exactly the c1 of the full twin written by the plain creators."""
    import oracle as O

    _build()
    r = subprocess.run([EXE, "roundtrip", str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    kmod = [int(x) for x in open(tmp_path / "key_moduli.txt").read().split()]
    n = 1 << 13
    ctx = O.Context(13, kmod)
    b = open(tmp_path / "ct_seeded.bin", "rb").read()
    end, f, c0, seed = _parse_ct(b)
    assert end == len(b) and seed is not None and f["size"] == 2
    t = open(tmp_path / "ct_twin.bin", "rb").read()
    _, ft, twin, tseed = _parse_ct(t)
    assert tseed is None and ft == f
    assert np.array_equal(c0[0], twin[0])
    assert np.array_equal(ctx.sample(seed, "uniform", f["L"]), twin[1])
    assert len(b) == len(t) - 8 * f["L"] * n + 81
    # relin keys: every digit record seeded; digit j's seed expands to the twin's c1 over all K primes
    kb = open(tmp_path / "relin_seeded.bin", "rb").read()
    kt = open(tmp_path / "relin_twin.bin", "rb").read()
    assert _header(kb) == len(kb) and _header(kt) == len(kt)
    dim1, dim2 = struct.unpack_from("<QQ", kb, 48)
    assert (dim1, dim2) == (1, len(kmod) - 1) and struct.unpack_from("<QQ", kt, 48) == (dim1, dim2)
    ob, ot = 64, 64
    for _ in range(dim2):
        ob, fb, c0b, sd = _parse_ct(kb, ob)
        ot, ft, twin, _ = _parse_ct(kt, ot)
        assert sd is not None and fb["L"] == len(kmod)
        assert np.array_equal(c0b[0], twin[0])
        assert np.array_equal(ctx.sample(sd, "uniform", len(kmod)), twin[1])
    assert ob == len(kb) and ot == len(kt)
