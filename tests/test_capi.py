"""CPU-side checks of the C ABI boundary (no GPU compute): libmhe.so loads, exports every
entry point include/mhe.h declares, and its host-only helpers agree with the oracle/KATs."""
import ctypes
import json
import os
import re

import pytest

import mhe
import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "mhe.h")).read()
    return sorted(set(re.findall(r"\b(mhe_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(mhe.LIB_PATH)
    names = declared_symbols()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and the Python binding binds exactly the declared surface
    assert set(mhe.SIGNATURES) == set(names)


def test_coeff_modulus_create_matches_oracle():
    for n, bits in [(1 << 16, [51] + [46] * 30 + [51] * 13 + [51]),
                    (1 << 16, [49] + [46] * 21 + [49] * 14 + [60]),
                    (1 << 12, [30, 40, 50, 60])]:
        assert mhe.coeff_modulus_create(n, bits) == O.coeff_modulus_create(n, bits)


def test_coeff_modulus_create_kats():
    kats = json.load(open(os.path.join(ROOT, "tests", "golden", "seal_kats.json")))["coeff_modulus_create"]
    for n, bits, want in kats["cases"]:
        assert mhe.coeff_modulus_create(n, bits) == want
    with pytest.raises(mhe.MheError):
        mhe.coeff_modulus_create(1 << 16, [61])


def test_galois_elt_from_step():
    kats = json.load(open(os.path.join(ROOT, "tests", "golden", "seal_kats.json")))["galois_elt_from_step"]
    for step, elt in kats["cases"]:
        assert mhe.galois_elt_from_step(kats["log_n"], step) == elt
    for step in (1, -1, 5, 1000, -32767, 0):
        assert mhe.galois_elt_from_step(16, step) == O.galois_elt_from_step(1 << 16, step)
    assert mhe.galois_elt_from_step(16, 1 << 15) == 0  # step count too large


def test_ctx_create_rejects_bad_chain_without_gpu_work():
    lib = mhe.lib()
    h = ctypes.c_void_p()
    bad = (ctypes.c_uint64 * 2)(12289, 15)  # 15 is not prime / not NTT friendly
    assert lib.mhe_ctx_create(ctypes.byref(h), 12, bad, 2, 0) == -1
    assert b"NTT-friendly" in lib.mhe_last_error()
    assert lib.mhe_ctx_create(ctypes.byref(h), 20, bad, 2, 0) == -1
