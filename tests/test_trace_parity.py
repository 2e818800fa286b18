"""Caller-sequence parity at ciphertext level: one multiplexed
convolution at 3 limbs (cnn/cnn_seal.cpp:284-530, whose top-level encryption of zero takes
add_inplace_reduced_error's unequal-level branch, SEAL/evaluator.cpp:312-362), one batch norm
(cnn_seal.cpp:531-576) and one ReLU polynomial (comp/SEALcomp.cpp:3-60, comp/SEALfunc.cpp:59-260)
run on the GPU through the seal:: surface with seeded keys (Blake2xbPRNGFactory {1..8}) and the
evaluator trace on (build/trace_caller_test, seal/trace.h); every recorded operation -- encodes,
rotations, plaintext products, reduced-error adds / subs / multiplies with their scale forcing,
rescales, relinearizations -- is then recomputed by the CPU oracle (tests/trace_replay.py over
oracle/evaluator.py) from the recorded inputs and must match word for word, scale for scale."""
import os
import subprocess

import pytest

from trace_replay import Replayer

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("log_n", [12, 16])
def test_conv_bn_relu_sequence_matches_oracle(tmp_path, log_n):
    d = tmp_path / f"trace{log_n}"
    d.mkdir()
    exe = os.path.join(ROOT, "build", "trace_caller_test")
    r = subprocess.run([exe, str(log_n), str(d), os.path.join(ROOT, "tests", "golden", "comp")], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    rp = Replayer(str(d))
    checked, counts = rp.replay()
    print(f"N=2^{log_n}: {checked} operations match the oracle: {counts}")
    # the sequence must have exercised the operations A11 / A19 / A20 name
    for op in ("rotate", "multiply_plain", "multiply_plain_add", "add_re", "sub_re", "mul_re", "rescale",
               "encode_for", "multiply_const"):
        assert counts.get(op, 0) > 0, f"{op} not exercised: {counts}"


@pytest.mark.parametrize("log_n,logn", [(12, 9), (12, 10)])
def test_sparse_bootstrap_matches_oracle(tmp_path, log_n, logn):
    """One sparse bootstrap_real_3 (Bootstrapper.cpp:3166-3236) at N = 2^12 on the ResNet chain shape,
    replayed op by op: modraise (:2894-2948), the subsum rotations, CoeffToSlot's three BSGS groups
    (sflinv_3, :2531; bsgs / rotated_bsgs_linear_transform, :1952-2085) with the reference-order LT
    diagonals, EvalMod (ModularReducer.cpp:61-80: the cosine heap polynomial of Polynomial.cpp:256-560,
    two double-angle steps, the linear arcsine), SlotToCoeff (sfl_half_3, :2453) and the final
    conjugate add -- every output word and scale equal to the oracle's."""
    d = tmp_path / f"boot{log_n}_{logn}"
    d.mkdir()
    exe = os.path.join(ROOT, "build", "trace_caller_test")
    r = subprocess.run([exe, str(log_n), str(d), os.path.join(ROOT, "tests", "golden", "comp"), "boot", str(logn)],
                       capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    rp = Replayer(str(d))
    checked, counts = rp.replay()
    print(f"N=2^{log_n}, logn {logn}: {checked} bootstrap operations match the oracle: {counts}")
    for op in ("modraise", "ntt_inv", "ntt_fwd", "rotate", "galois", "encode_for", "multiply_plain",
               "multiply_plain_add", "rescale", "mul_re", "add_re", "add_const", "multiply_const"):
        assert counts.get(op, 0) > 0, f"{op} not exercised: {counts}"


@pytest.mark.parametrize("logn", [12, 14])
def test_sparse_bootstrap_resnet_shape_matches_oracle(tmp_path, logn):
    """The bootstraps ResNet runs, at their own shape: bootstrap_real_3
    at N = 2^16 on the 31 + 1 prime chain (cnn/infer_seal.cpp:288-316) with logn 12 sparse slots, the
    third bootstrapper of ResNet-20, and logn 14, the first and largest one (76 rotations, its own
    giant-step split, COMMON/func.cpp:203) (Bootstrapper.cpp:3166-3236, called from
    infer_seal.cpp:340-342,486-533), replayed op by op through the oracle on 16 host threads; every
    word and scale must be equal."""
    import shutil

    d = tmp_path / f"boot16_{logn}"
    d.mkdir()
    exe = os.path.join(ROOT, "build", "trace_caller_test")
    r = subprocess.run([exe, "16", str(d), os.path.join(ROOT, "tests", "golden", "comp"), "boot", str(logn)],
                       capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    size = sum(f.stat().st_size for f in d.iterdir())
    rp = Replayer(str(d))
    checked, counts = rp.replay(threads=16)
    print(f"N=2^16, logn {logn}: {checked} bootstrap operations ({size / 1e9:.1f} GB of trace) match the oracle: {counts}")
    for op in ("modraise", "rotate", "galois", "multiply_plain", "rescale", "mul_re", "add_re"):
        assert counts.get(op, 0) > 0, f"{op} not exercised: {counts}"
    shutil.rmtree(d, ignore_errors=True)


@pytest.mark.parametrize("log_n", [12, 16])
def test_downsample_add_avgpool_fc_match_oracle(tmp_path, log_n):
    """The ResNet layers the conv / BN / ReLU trace does not reach, in network order
    (cnn/infer_seal.cpp:520-560): multiplexed_parallel_downsampling_seal (cnn/cnn_seal.cpp:610-679),
    cnn_add_seal (:593-609), averagepooling_seal_scale (:680-746) and matrix_multiplication_seal
    (:747-787) -- every operation word for word and scale for scale against the oracle."""
    d = tmp_path / f"layers{log_n}"
    d.mkdir()
    exe = os.path.join(ROOT, "build", "trace_caller_test")
    r = subprocess.run([exe, str(log_n), str(d), os.path.join(ROOT, "tests", "golden", "comp"), "layers"],
                       capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    rp = Replayer(str(d))
    checked, counts = rp.replay()
    print(f"N=2^{log_n}: {checked} layer operations match the oracle: {counts}")
    for op in ("rotate", "multiply_plain", "add_re", "rescale", "encode_for"):
        assert counts.get(op, 0) > 0, f"{op} not exercised: {counts}"
