"""GPT-2 layer over the SEAL surface (include/mhe_gpt2.h, fhe-gpt-2_amd/seal/gpt2.cpp) -- config C5's
pieces: Chebyshev basis, composite sign, GELU p/q, exp, Goldschmidt inverse, quickSum and the
row-packed encrypted matmul (gpt2_ckks/gpt2-ckks/single-key/gpt2/).  The GPU test runs the
reference's own doctest cases with their expected values (gpt2_ckks/run/run_approx_test.cpp) and
checks every approximation over all 32768 slots against its plain-double restatement within 1e-3
(tests/cpp/gpt2_test.cpp)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "fhe-gpt-2_amd")


def _build():
    subprocess.check_call(["make", "-s", "-C", os.path.join(PKG, "seal"), "all", "test"])


def test_gpt2_symbols_exported():
    _build()
    out = subprocess.check_output(["nm", "-DC", "--defined-only", os.path.join(PKG, "libmhe_seal.so")], text=True)
    for sym in ("gpt2::build_cheby_basis", "gpt2::compute_sign_f", "gpt2::compute_sign_g", "gpt2::sign_function",
                "gpt2::compute_gelu_p", "gpt2::compute_gelu_q", "gpt2::compute_gelu", "gpt2::compute_exp",
                "gpt2::compute_inverse", "gpt2::quickSum", "gpt2::mask_out", "gpt2::pack_from_row",
                "gpt2::row_matrix_multiplication_seal", "gpt2::compute_smax",
                "gpt2::fakeBootstrap", "gpt2::taylor_expand", "gpt2::compute_inv_sqrt", "gpt2::compute_layernorm",
                "gpt2::surefire_rotate", "gpt2::attn_proj_row_seal", "gpt2::attn_proj_col_seal",
                "gpt2::qk_matmul", "gpt2::sv_matmul",
                "gpt2::batch_matmul", "gpt2::qk_matmul_col", "gpt2::cipher_plain_128_128",
                "gpt2::bootstrap", "gpt2::init_bootstrap", "gpt2::computeMax", "gpt2::quickMax",
                "gpt2::compute_softmax"):
        assert sym in out, sym


@pytest.mark.gpu
def test_gpt2_approximations_end_to_end():
    _build()
    r = subprocess.run([os.path.join(ROOT, "build", "gpt2_test")], capture_output=True, text=True, timeout=600)
    print(r.stdout)
    print(r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
@pytest.mark.skipif(not os.environ.get("MHE_LONG"), reason="about 3 minutes of on-the-spot keygen; set MHE_LONG=1")
def test_gpt2_attention_matmuls():
    """qk_matmul / sv_matmul (MatrixMul.cpp:480-584): 16384 + 8192 surefire_rotate keys."""
    _build()
    env = dict(os.environ, GPT2_QKV="1")
    r = subprocess.run([os.path.join(ROOT, "build", "gpt2_test")], capture_output=True, text=True, timeout=900, env=env)
    print(r.stdout)
    print(r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
