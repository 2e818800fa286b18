"""The SEAL-compatible C++ surface (fhe-gpt-2_amd/include/seal/seal.h, libmhe_seal.so):
the CPU side checks that it loads; the GPU side runs tests/cpp/seal_api_test.cpp -- the
reference's CKKS GoogleTest scenarios written against the same API -- end to end."""
import ctypes
import os
import sys
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "fhe-gpt-2_amd")
DRIVER = os.path.join(ROOT, "build", "seal_api_test")


def _build():
    subprocess.check_call(["make", "-s", "-C", os.path.join(PKG, "seal"), "all", "test"])


def test_seal_library_loads():
    _build()
    lib = ctypes.CDLL(os.path.join(PKG, "libmhe_seal.so"))
    # mangled C++ entry points of the drop-in (a few representative ones)
    out = subprocess.check_output(["nm", "-D", "--defined-only", os.path.join(PKG, "libmhe_seal.so")], text=True)
    for sym in ("seal::Evaluator::multiply_inplace", "seal::Evaluator::relinearize_inplace",
                "seal::Evaluator::rescale_to_next", "seal::Evaluator::rotate_vector_inplace",
                "seal::Evaluator::add_inplace_reduced_error", "seal::CKKSEncoder::encode",
                "seal::KeyGenerator::create_galois_keys"):
        dem = subprocess.check_output(["c++filt"], input=out, text=True)
        assert sym in dem, sym
    assert lib is not None


@pytest.mark.gpu
def test_cnn_layers_end_to_end():
    """Multiplexed-packing CNN layers (include/mhe_cnn.h, cnn_seal.cpp semantics) on encrypted
    tensors vs the same layers in plain doubles (tests/cpp/cnn_test.cpp)."""
    _build()
    r = subprocess.run([os.path.join(ROOT, "build", "cnn_test")], capture_output=True, text=True, timeout=900)
    print(r.stdout)
    print(r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_approx_relu_end_to_end():
    """Approximate ReLU by the reference's minimax composite polynomial (alpha 13, degrees
    {15,15,27}, odd baby-step trees; include/mhe_comp.h) on the GPU vs max(x, 0)."""
    _build()
    env = dict(os.environ, MHE_COMP_DIR=os.path.join(ROOT, "tests", "golden", "comp"))
    r = subprocess.run([os.path.join(ROOT, "build", "comp_test")], capture_output=True, text=True, timeout=900,
                       env=env)
    print(r.stdout)
    print(r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr


def test_bootstrapping_host_math():
    """CPU: merged CoeffToSlot/SlotToCoeff diagonals vs the sparse canonical embedding, cosine fit
    error on the union of intervals, Chebyshev heap identities (tests/cpp/boot_host_test.cpp)."""
    _build()
    r = subprocess.run([os.path.join(ROOT, "build", "boot_host_test")], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("logn", ["14", "15"], ids=["sparse_logn14", "full_slots_logn15"])
def test_bootstrapping_end_to_end(logn):
    """CKKS bootstrapping (include/mhe_boot.h, ckks_bootstrapping/Bootstrapper.cpp semantics) in the
    reference ResNet setting: N=2^16, 31 data limbs, 1 limb -> refreshed; logn 14 sparse slots
    (bootstrap_sparse_real_3) and all 2^15 slots (bootstrap_full_real_3, the GPT-2 path's
    bootstrap_3); decrypted output within 1e-3 of the message (tests/cpp/boot_test.cpp)."""
    _build()
    r = subprocess.run([os.path.join(ROOT, "build", "boot_test"), logn, "2"], capture_output=True, text=True,
                       timeout=900)
    print(r.stdout)
    print(r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_resnet20_end_to_end():
    """Encrypted ResNet-20 CIFAR-10 (include/mhe_resnet.h, cnn/infer_seal.cpp semantics: multiplexed
    conv/BN, approximate ReLU, 18 sparse-slot bootstraps, average pooling, FC) with the reference's
    pretrained parameters on a seeded synthetic image and fresh keys; decrypted logits vs the plain
    network with the encrypted network's own minimax-composite ReLU (the encryption's error alone)
    and, as a sanity check, vs the exact-ReLU network, each within 8% of the largest logit
    (tests/cpp/resnet_test.cpp)."""
    _build()
    r = subprocess.run([os.path.join(ROOT, "build", "resnet_test"),
                        os.path.join(ROOT, "tests", "golden", "resnet", "resnet20_params.bin"),
                        os.path.join(ROOT, "tests", "golden", "comp"), "1"],
                       capture_output=True, text=True, timeout=900)
    print(r.stdout)
    print(r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_resnet20_fiber_batch_bench_shape_words_equal_alone():
    """The batch shape the bench times: 16 ResNet-20 images as 2 host threads x
    8 fibers, so merged launches carry the full MHE_MAXB = 8 entries, hoisted rotations on as the
    bench runs them (and off, and on with the classic-path check) -- every image's output ciphertext
    words equal the same image run alone (cnn/infer_seal.cpp:404-577 defines each image by its own
    run; tests/cpp/resnet_test.cpp fibercheck)."""
    _build()
    r = subprocess.run([os.path.join(ROOT, "build", "resnet_test"),
                        os.path.join(ROOT, "tests", "golden", "resnet", "resnet20_params.bin"),
                        os.path.join(ROOT, "tests", "golden", "comp"), "fibercheck", "16", "2", "8"],
                       capture_output=True, text=True, timeout=900)
    print(r.stdout)
    print(r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("0 of 16 digests differ from alone") == 3, r.stdout


@pytest.mark.gpu
def test_resnet20_fiber_batch_words_equal_alone():
    """The bench's batched ResNet mode against the reference's per-image definition
    (cnn/infer_seal.cpp:404-577 runs every image on its own): 4 ResNet-20 images as 2 host threads x
    2 fibers (seal::FiberBatch: merged rotations / relinearizations / rescales, coalesced
    elementwise launches) must each give the output ciphertext words of the same image run alone,
    with hoisted rotations off, on with a check (every hoisted rotation also recomputed by the classic
    path, word for word) and on as the bench runs it (tests/cpp/resnet_test.cpp fibercheck).
    Keys come from the runner's reproducible seed sequence and every encryption from its base seed
    (seal.h Blake2xbSeedSequence), so each image's words do not depend on thread or fiber order."""
    _build()
    r = subprocess.run([os.path.join(ROOT, "build", "resnet_test"),
                        os.path.join(ROOT, "tests", "golden", "resnet", "resnet20_params.bin"),
                        os.path.join(ROOT, "tests", "golden", "comp"), "fibercheck", "4", "2", "2"],
                       capture_output=True, text=True, timeout=900)
    print(r.stdout)
    print(r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("0 of 4 digests differ from alone") == 3, r.stdout


def test_resnet_params_fixture():
    """The packed parameter fixture has ResNet-20's 271098 values in import_parameters_cifar10
    order (cnn/infer_seal.cpp:3-100): 19 conv weight tensors, 19 x 4 batch-norm vectors, FC."""
    import numpy as np

    v = np.fromfile(os.path.join(ROOT, "tests", "golden", "resnet", "resnet20_params.bin"), dtype="<f8")
    conv = 9 * 3 * 16 + 3 * 2 * 9 * 16 * 16 + 9 * 16 * 32 + 9 * 32 * 32 + 2 * 2 * 9 * 32 * 32 + 9 * 32 * 64 \
        + 9 * 64 * 64 + 2 * 2 * 9 * 64 * 64
    bnv = 4 * (16 + 6 * 16 + 6 * 32 + 6 * 64)
    assert v.size == conv + bnv + 640 + 10
    assert np.isfinite(v).all()
    # running variances are positive
    off = conv
    sizes = [16] + [16] * 6 + [32] * 6 + [64] * 6
    for c in sizes:
        var = v[off + 2 * c: off + 3 * c]
        assert (var > 0).all()
        off += 4 * c


@pytest.mark.gpu
def test_resnet110_end_to_end():
    """Config C4's network: encrypted ResNet-110 CIFAR-10 (end_num 17: 54 residual blocks, 108
    sparse-slot bootstraps) with the reference's pretrained ResNet-110 parameters
    (tests/golden/resnet/resnet110_params.d7) on one seeded synthetic image; decrypted logits vs the
    plain network within 8% of the largest logit (tests/cpp/resnet_test.cpp)."""
    _build()
    r = subprocess.run([os.path.join(ROOT, "build", "resnet_test"),
                        os.path.join(ROOT, "tests", "golden", "resnet", "resnet110_params.d7"),
                        os.path.join(ROOT, "tests", "golden", "comp"), "1", "110"],
                       capture_output=True, text=True, timeout=900)
    print(r.stdout)
    print(r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr


def test_resnet110_params_fixture():
    """The lossless 4-byte ".d7" packing of ResNet-110's parameters: the C++ loader
    (load_resnet_params_bin) and the Python decoder of make_resnet_params.py agree value for value
    (count and left-to-right sum printed by `resnet_test ... -1 110`, no GPU); where the reference
    is mounted, the decoded values equal the reference's text parsed as doubles."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_resnet_params as m

    path = os.path.join(ROOT, "tests", "golden", "resnet", "resnet110_params.d7")
    v = m.unpack_d7(open(path, "rb").read())
    conv = 9 * 3 * 16 + 18 * 2 * 9 * 16 * 16 + 9 * 16 * 32 + 9 * 32 * 32 + 17 * 2 * 9 * 32 * 32 \
        + 9 * 32 * 64 + 9 * 64 * 64 + 17 * 2 * 9 * 64 * 64
    assert v.size == conv + 4 * (16 + 36 * (16 + 32 + 64)) + 640 + 10
    _build()
    r = subprocess.run([os.path.join(ROOT, "build", "resnet_test"), path, "unused", "-1", "110"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"params: {v.size} values, sum {sum(v.tolist())!r}" in r.stdout, r.stdout
    src = "/root/reference/pretrained_parameters/resnet110_new"
    if os.path.isdir(src):
        w = np.array([float(t) for t in open(os.path.join(src, "conv1_weight.txt")).read().split()[:432]])
        assert np.array_equal(v[:432], w)
        b = np.array([float(t) for t in open(os.path.join(src, "linear_bias.txt")).read().split()[:10]])
        assert np.array_equal(v[-10:], b)


@pytest.mark.gpu
def test_seal_api_end_to_end():
    _build()
    r = subprocess.run([DRIVER], capture_output=True, text=True, timeout=600)
    print(r.stdout)
    print(r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed" in r.stdout


def _consumer(tmp):
    _build()
    bdir = os.path.join(tmp, "consumer")
    subprocess.check_call(["cmake", "-S", os.path.join(ROOT, "tests", "cpp", "consumer"), "-B", bdir,
                           "-DCMAKE_PREFIX_PATH=" + PKG, "-DCMAKE_BUILD_TYPE=Release"],
                          stdout=subprocess.DEVNULL)
    subprocess.check_call(["cmake", "--build", bdir], stdout=subprocess.DEVNULL)
    return os.path.join(bdir, "consumer")


def test_cmake_package_consumer_builds(tmp_path):
    """find_package(SEAL 3.6 REQUIRED) + SEAL::seal resolves to this package (the reference's
    CMake integration, cnn_ckks/CMakeLists.txt:11,60) and a caller compiles and links."""
    exe = _consumer(str(tmp_path))
    assert os.path.exists(exe)


@pytest.mark.gpu
def test_cmake_package_consumer_runs(tmp_path):
    exe = _consumer(str(tmp_path))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_cnn_cli_stage_levels_match_reference(tmp_path):
    """Config C1 plumbing: `cnn 20 10 0 0` (cnn_ckks/run/run_cnn.cpp) writes
    ../../result/resnet20_cifar10_image0.txt and resnet20_cifar10_label_0_0 in the reference's format
    (cnn/infer_seal.cpp:408-582).  Its stage sequence -- every logged op with its remaining level and
    printed scale -- must equal the reference's own run on image 0 (tests/golden/resnet/
    resnet20_image0_stages.json, extracted by make_resnet_stage_fixture.py).  Values differ: the
    reference's input pixels are not in its tree, so the image is synthetic."""
    import json

    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from make_resnet_stage_fixture import parse

    _build()
    run_dir = tmp_path / "cnn_ckks" / "build"
    run_dir.mkdir(parents=True)
    (tmp_path / "result").mkdir()
    env = dict(os.environ, MHE_RESNET_PARAMS=os.path.join(ROOT, "tests", "golden", "resnet", "resnet20_params.bin"),
               MHE_COMP_DIR=os.path.join(ROOT, "tests", "golden", "comp"))
    r = subprocess.run([os.path.join(ROOT, "build", "cnn"), "20", "10", "0", "0"], cwd=run_dir, env=env,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "model: ResNet-20" in r.stdout and "inferred label:" in r.stdout
    log = (tmp_path / "result" / "resnet20_cifar10_image0.txt").read_text()
    got = parse(log)
    want = json.load(open(os.path.join(ROOT, "tests", "golden", "resnet", "resnet20_image0_stages.json")))["stages"]
    assert [(s["layer"], s["op"]) for s in got] == [(s["layer"], s["op"]) for s in want]
    for g, w in zip(got, want):
        assert (g["level"], g["scale"]) == (w["level"], w["scale"]), (g, w)
    share = (tmp_path / "result" / "resnet20_cifar10_label_0_0").read_text()
    assert share.startswith("image_id: 0, image label: -1, inferred label: ") and "all threads time :" in share
