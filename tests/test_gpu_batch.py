"""GPU parity of the batched launches (include/mhe.h mhe_apply_galois_batch / mhe_rescale_batch /
mhe_switch_key_batch): `count` independent operations of one level in one launch per kernel must
give, entry for entry, the same words as the oracle's single-ciphertext restatement of
apply_galois_inplace / divide_and_round_q_last_ntt_inplace / switch_key_inplace
(SEAL/evaluator.cpp:2120-2222, 2281-2525; SEAL/util/rns.cpp:737-808).  Batches larger than one
launch's 8 entries run in groups, so 9 and 11 cover the split."""
import numpy as np
import pytest

import mhe
import oracle as O
from test_gpu_parity import RESNET_BITS, SMALL_BITS, Chain

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def small():
    return Chain(12, SMALL_BITS, seed=11)


@pytest.fixture(scope="module")
def resnet():
    return Chain(16, RESNET_BITS, seed=12)


class hoisting:
    """Hoisted rotations on for the block (mhe_ctx_set_hoist; on is also the context default) with
    the engine's own check (every hoisted rotation recomputed by the classic path and compared).
    On exit: the hoisted key-MAC kernels must have run (mhe_hoist_stats) and the check must have
    found no differing word; the context's previous setting is restored, so the tests after this
    one see the same default whatever the order."""

    def __init__(self, eng, min_rotations=1):
        self.eng, self.min_rotations = eng, min_rotations

    def __enter__(self):
        self.saved = self.eng.hoist()
        self.eng.set_hoist(True, check=True)
        assert self.eng.hoist() == (True, True)
        self.eng.hoist_stats(reset=True)
        return self

    def __exit__(self, *exc):
        self.eng.synchronize()
        rot, mac, bad = self.eng.hoist_stats(reset=True)
        self.eng.set_hoist(*self.saved)
        if exc[0] is None:
            assert rot >= self.min_rotations and mac >= 1, (rot, mac)
            assert bad == 0, f"{bad} words of hoisted rotations differ from the classic path"
        return False


def truncated(key, L):
    """The level-L slice of a key: L digits, data primes 0..L-1 and the special prime."""
    return np.ascontiguousarray(np.concatenate([key[:L, :, :L], key[:L, :, -1:]], axis=2))


@pytest.mark.parametrize("L", [1, 3, 7])
@pytest.mark.parametrize("count", [1, 3, 8, 11])
def test_rotate_batch_one_input(small, L, count):
    """The conv / BSGS baby-step shape: one input rotated by `count` different steps."""
    ch = small
    ct = ch.rand(2, L, ch.n)
    steps = [1, -1, 3, 100, 0, 7, -5, 64, 2, 9, 31][:count]
    elts = [mhe.galois_elt_from_step(ch.log_n, s) for s in steps]
    keys = [ch.rand_key() for _ in steps]
    dkeys = [ch.up(k if i % 2 else truncated(k, L)) for i, k in enumerate(keys)]  # full and level-truncated
    src = ch.up(ct)
    outs = ch.eng.apply_galois_batch([src] * count, elts, dkeys)
    for i in range(count):
        assert np.array_equal(ch.down(outs[i]), ch.oc.apply_galois(ct, elts[i], keys[i])), f"entry {i} step {steps[i]}"
    assert np.array_equal(ch.down(src), ct)  # inputs untouched


@pytest.mark.parametrize("count", [2, 9])
def test_rotate_batch_many_inputs(small, count):
    """The multi-image / giant-step shape: different inputs, the same or different keys."""
    ch = small
    L = 5
    key = ch.rand_key()
    cts = [ch.rand(2, L, ch.n) for _ in range(count)]
    elts = [mhe.galois_elt_from_step(ch.log_n, 1 + (i % 3)) for i in range(count)]
    dk = ch.up(key)
    outs = ch.eng.apply_galois_batch([ch.up(c) for c in cts], elts, [dk] * count)
    for i in range(count):
        assert np.array_equal(ch.down(outs[i]), ch.oc.apply_galois(cts[i], elts[i], key))


def test_rotate_batch_prepared_keys_n16(resnet):
    """N = 2^16 on the ResNet chain with prepared keys (residues as doubles): the packed ModUp intermediate and
    key planes per entry, at a bootstrap-like level."""
    ch = resnet
    L = 6
    ct = ch.rand(2, L, ch.n)
    steps = [1, 2, 4, 8]
    elts = [mhe.galois_elt_from_step(ch.log_n, s) for s in steps]
    keys = [truncated(ch.rand_key(digits=L), L) for _ in steps]
    # both prepared formats in one call (doubles, 48-bit planes, alternating)
    dkeys = [ch.eng.key_prepare(ch.up(k), 1 + i % 2) for i, k in enumerate(keys)]
    outs = ch.eng.apply_galois_batch([ch.up(ct)] * len(steps), elts, dkeys)
    full = [np.zeros((L, 2, ch.K, ch.n), np.uint64) for _ in keys]
    for f, k in zip(full, keys):  # the truncated slice inside a full-shape key for the oracle
        f[:, :, :L] = k[:, :, :L]
        f[:, :, -1] = k[:, :, -1]
    for i in range(len(steps)):
        assert np.array_equal(ch.down(outs[i]), ch.oc.apply_galois(ct, elts[i], full[i]))


def with_zero_coeffs(ch, L, zeros):
    """A ciphertext whose c1 (coefficient form) has zero coefficients: `zeros` random slots >= 1 per
    limb, "slot0" (slot 0 only, never negated by a rotation) or "all".  A hoisted rotation's
    identity fails at a zero moved to a negated slot (csrc/hoist.h), so the engine must take the
    classic path for such an input, decided on the device."""
    ct = ch.rand(2, L, ch.n)
    c1 = ch.rand(L, ch.n)
    if zeros == "all":
        c1[:] = 0
    elif zeros == "slot0":
        c1[:, 0] = 0
    else:
        for l in range(L):
            c1[l, ch.rng.choice(np.arange(1, ch.n), zeros, replace=False)] = 0
    ct[1] = ch.oc.ntt(c1)
    return ct


@pytest.mark.parametrize("zeros", [0, "slot0", 1, 7, "all"])
def test_rotate_batch_hoisted_zero_coefficients(small, zeros):
    """One input rotated 4 ways (the hoisted path: one shared ModUp) with zero coefficients in its
    c1: every output still equals the oracle's one-at-a-time apply_galois."""
    ch = small
    L = 4
    ct = with_zero_coeffs(ch, L, zeros)
    steps = [1, 3, -2, 17]
    elts = [mhe.galois_elt_from_step(ch.log_n, s) for s in steps]
    keys = [ch.rand_key() for _ in steps]
    with hoisting(ch.eng, len(steps)):
        outs = ch.eng.apply_galois_batch([ch.up(ct)] * len(steps), elts, [ch.up(k) for k in keys])
    for i in range(len(steps)):
        assert np.array_equal(ch.down(outs[i]), ch.oc.apply_galois(ct, elts[i], keys[i])), f"step {steps[i]}"


def test_rotate_batch_hoisted_mixed(small):
    """10 inputs in one call -- 8 rotated 2-4 ways (hoisted, in two passes of at most 8 inputs), two
    rotated once (the classic path), one with zero coefficients among them -- shared and distinct
    keys, full and level-truncated."""
    ch = small
    L = 5
    shared = ch.rand_key()
    cts = [with_zero_coeffs(ch, L, 3) if i == 4 else ch.rand(2, L, ch.n) for i in range(10)]
    srcs = [ch.up(c) for c in cts]
    reps = [2, 3, 4, 2, 3, 1, 2, 4, 1, 2]
    ins, elts, keys, dkeys, which = [], [], [], [], []
    for i, r in enumerate(reps):
        for k in range(r):
            step = [1, 2, 5, -3][k]
            key = shared if (i + k) % 2 else ch.rand_key()
            ins.append(srcs[i])
            elts.append(mhe.galois_elt_from_step(ch.log_n, step))
            keys.append(key)
            dkeys.append(ch.up(key if k % 2 else truncated(key, L)))
            which.append(i)
    with hoisting(ch.eng, len(ins) - 2):
        outs = ch.eng.apply_galois_batch(ins, elts, dkeys)
    for j in range(len(ins)):
        want = ch.oc.apply_galois(cts[which[j]], elts[j], keys[j])
        assert np.array_equal(ch.down(outs[j]), want), f"entry {j} (input {which[j]})"
    for c, s in zip(cts, srcs):
        assert np.array_equal(ch.down(s), c)  # inputs untouched


@pytest.mark.parametrize("L", [1, 6])
def test_rotate_batch_hoisted_shared_keys(small, L):
    """4 inputs rotated by the same 3 keys (a FiberBatch's baby steps): the keys' mask sums are taken
    once per key (k_hoist_kc); one input has zero coefficients, one key is level-truncated."""
    ch = small
    cts = [ch.rand(2, L, ch.n), ch.rand(2, L, ch.n), with_zero_coeffs(ch, L, 4), ch.rand(2, L, ch.n)]
    steps = [1, -4, 9]
    elts = [mhe.galois_elt_from_step(ch.log_n, s) for s in steps]
    keys = [ch.rand_key() for _ in steps]
    dkeys = [ch.up(truncated(k, L) if i == 1 else k) for i, k in enumerate(keys)]
    srcs = [ch.up(c) for c in cts]
    ins = [s for s in srcs for _ in steps]
    with hoisting(ch.eng, len(ins)):
        outs = ch.eng.apply_galois_batch(ins, elts * len(cts), dkeys * len(cts))
    for j in range(len(ins)):
        want = ch.oc.apply_galois(cts[j // 3], elts[j % 3], keys[j % 3])
        assert np.array_equal(ch.down(outs[j]), want), f"input {j // 3} step {steps[j % 3]}"


def test_rotate_batch_hoisted_n16(resnet):
    """N = 2^16, ResNet chain at 12 limbs, prepared keys: 3 inputs x 3 rotations (BSGS baby steps of
    three images), one input with zero coefficients."""
    ch = resnet
    L = 12
    cts = [ch.rand(2, L, ch.n), with_zero_coeffs(ch, L, 2), ch.rand(2, L, ch.n)]
    steps = [1, 2, 3]
    keys = [truncated(ch.rand_key(digits=L), L) for _ in steps]
    dkeys = [ch.eng.key_prepare(ch.up(k), 1 + i % 2) for i, k in enumerate(keys)]  # mixed formats
    full = [np.zeros((L, 2, ch.K, ch.n), np.uint64) for _ in keys]
    for f, k in zip(full, keys):
        f[:, :, :L] = k[:, :, :L]
        f[:, :, -1] = k[:, :, -1]
    elts = [mhe.galois_elt_from_step(ch.log_n, s) for s in steps]
    srcs = [ch.up(c) for c in cts]
    ins = [s for s in srcs for _ in steps]
    with hoisting(ch.eng, 9):
        outs = ch.eng.apply_galois_batch(ins, elts * 3, dkeys * 3)
    for j in range(9):
        want = ch.oc.apply_galois(cts[j // 3], elts[j % 3], full[j % 3])
        assert np.array_equal(ch.down(outs[j]), want), f"input {j // 3} step {steps[j % 3]}"


@pytest.mark.parametrize("zero_input", [None, 3])
def test_rotate_batch_hoisted_fiber_bsgs_shape(resnet, zero_input):
    """The shape the ResNet FiberBatch runs in its bootstraps: 8 inputs (the images of
    2 threads x 4 fibers share nothing, one thread's 4 are merged -- here all 8) x 7 baby-step
    rotations sharing the 7 keys (k_ks_hoist_mac_sh, R = 7, one item per lane group), N = 2^16 at
    24 limbs, prepared level-truncated keys, optionally one input with zero coefficients (its
    rotations take the classic path inside the same launch sequence).  Every output equals the
    engine's classic path (hoisting off), and two entries equal the oracle."""
    ch = resnet
    L = 24
    steps = [1, 2, 3, 4, 5, 6, 7]
    keys = [truncated(ch.rand_key(digits=L), L) for _ in steps]
    # the zero-input case with mixed key formats (the shared kernel's per-row format), the other
    # with the default
    dkeys = [ch.eng.key_prepare(ch.up(k), (1 + i % 2) if zero_input is not None else None) for i, k in enumerate(keys)]
    cts = [with_zero_coeffs(ch, L, 2) if i == zero_input else ch.rand(2, L, ch.n) for i in range(8)]
    srcs = [ch.up(c) for c in cts]
    elts = [mhe.galois_elt_from_step(ch.log_n, s) for s in steps]
    ins = [s for s in srcs for _ in steps]
    with hoisting(ch.eng, len(ins)):
        outs = ch.eng.apply_galois_batch(ins, elts * 8, dkeys * 8)
    saved = ch.eng.hoist()
    ch.eng.set_hoist(False)  # the classic path, explicitly
    try:
        classic = ch.eng.apply_galois_batch(ins, elts * 8, dkeys * 8)
    finally:
        ch.eng.set_hoist(*saved)
    for j in range(len(ins)):
        assert np.array_equal(ch.down(outs[j]), ch.down(classic[j])), f"input {j // 7} step {steps[j % 7]}"
    full = [np.zeros((L, 2, ch.K, ch.n), np.uint64) for _ in keys]
    for f, k in zip(full, keys):
        f[:, :, :L] = k[:, :, :L]
        f[:, :, -1] = k[:, :, -1]
    for j in (5, 7 * (zero_input or 0) + 3):
        want = ch.oc.apply_galois(cts[j // 7], elts[j % 7], full[j % 7])
        assert np.array_equal(ch.down(outs[j]), want), f"input {j // 7} step {steps[j % 7]} vs oracle"


@pytest.mark.parametrize("size", [1, 2, 3])
@pytest.mark.parametrize("count", [1, 5, 9])
def test_rescale_batch(small, size, count):
    ch = small
    L = 6
    cts = [ch.rand(size, L, ch.n) for _ in range(count)]
    outs = ch.eng.rescale_batch([ch.up(c) for c in cts])
    for c, o in zip(cts, outs):
        assert np.array_equal(ch.down(o), ch.oc.rescale(c))


@pytest.mark.parametrize("L", [1, 4])
def test_switch_key_batch(small, L):
    ch = small
    count = 3
    keys = [ch.rand_key() for _ in range(count)]
    cts = [ch.rand(2, L, ch.n) for _ in range(count)]
    tgs = [ch.rand(L, ch.n) for _ in range(count)]
    dct = [ch.up(c) for c in cts]
    ch.eng.switch_key_batch(dct, [ch.up(t) for t in tgs], [ch.up(k) for k in keys])
    for i in range(count):
        assert np.array_equal(ch.down(dct[i]), ch.oc.switch_key(cts[i], tgs[i], keys[i]))


@pytest.mark.parametrize("count", [1, 3, 8, 11])
def test_hmult_batch(small, count):
    """mhe_hmult_batch: independent HMults sharing the relinearization key (the XCD-grouped key
    stream of k_ks_row_mac) equal the oracle's HMult entry for entry, squares included."""
    ch = small
    L = ch.K - 1
    key = ch.rand_key()
    a = [ch.rand(2, L, ch.n) for _ in range(count)]
    b = [ch.rand(2, L, ch.n) for _ in range(count)]
    da = [ch.up(x) for x in a]
    db = [da[i] if i % 4 == 3 else ch.up(b[i]) for i in range(count)]  # every 4th entry a square
    outs = ch.eng.hmult_batch(da, db, ch.up(key))
    for i in range(count):
        want = ch.oc.hmult(a[i], a[i] if i % 4 == 3 else b[i], key)
        assert np.array_equal(ch.down(outs[i]), want), i


@pytest.mark.parametrize("prepared", [0, 1, 2], ids=["seal", "doubles", "pack48"])
def test_hmult_batch_resnet_size(resnet, prepared):
    """N = 2^16 (the grid where every tile count is a multiple of 8): 9 HMults in one call (8 + 1)
    equal one-by-one mhe_hmult, with SEAL's key layout and both prepared key formats."""
    ch = resnet
    L = 6
    key = ch.up(truncated(ch.rand_key(), L))
    if prepared:
        key = ch.eng.key_prepare(key, prepared)
    a = [ch.up(ch.rand(2, L, ch.n)) for _ in range(9)]
    b = [ch.up(ch.rand(2, L, ch.n)) for _ in range(9)]
    outs = ch.eng.hmult_batch(a, b, key)
    for i in range(9):
        assert np.array_equal(ch.down(outs[i]), ch.down(ch.eng.hmult(a[i], b[i], key))), i


def test_switch_key_batch_shared_key(small):
    """A batched key switch whose entries all read one key (XCD-grouped entries) equals the oracle."""
    ch = small
    L = 3
    key = ch.rand_key()
    dkey = ch.up(key)
    cts = [ch.rand(2, L, ch.n) for _ in range(8)]
    tgs = [ch.rand(L, ch.n) for _ in range(8)]
    dct = [ch.up(c) for c in cts]
    ch.eng.switch_key_batch(dct, [ch.up(t) for t in tgs], [dkey] * 8)
    for i in range(8):
        assert np.array_equal(ch.down(dct[i]), ch.oc.switch_key(cts[i], tgs[i], key))


def test_batch_errors(small):
    ch = small
    L = 3
    a = ch.up(ch.rand(2, L, ch.n))
    key = ch.up(ch.rand_key())
    elt = mhe.galois_elt_from_step(ch.log_n, 1)
    with pytest.raises(mhe.MheError, match="same value"):
        ch.eng.apply_galois_batch([a], [elt], [key], outs=[a])  # out aliases in
    o = ch.eng.empty(2, L, ch.n)
    with pytest.raises(mhe.MheError, match="same value"):
        ch.eng.apply_galois_batch([a, a], [elt, elt], [key, key], outs=[o, o])  # two outputs alias
    with pytest.raises(mhe.MheError, match="Galois element"):
        ch.eng.apply_galois_batch([a], [4], [key])
    with pytest.raises(mhe.MheError):
        ch.eng.rescale_batch([a], outs=[a])
    with pytest.raises(mhe.MheError, match="distinct"):
        ch.eng.hmult_batch([a, a], [a, a], key, outs=[o, o])


def test_batch_overlap_errors(small):
    """Entries of one batch run inside the same kernels, so an output may share no word with another
    entry's operand or output (partial overlaps, not just equal pointers, are refused
    before any launch); an output over its own operands stays allowed where one call allows it."""
    ch = small
    L = 4
    n = ch.n
    key = ch.up(ch.rand_key())
    big = ch.eng.empty(6, L, n)  # one allocation, sliced so that ranges overlap partially
    x = ch.up(ch.rand(2, L, n))
    y = ch.up(ch.rand(2, L, n))
    # rescale: out[0] overlaps the second half of in[1]
    in1 = big[0:2]
    out0 = big.view(-1)[(2 * L - 1) * n:(2 * L - 1) * n + 2 * (L - 1) * n].view(2, L - 1, n)
    with pytest.raises(mhe.MheError, match="alias"):
        ch.eng.rescale_batch([x, in1], outs=[out0, ch.eng.empty(2, L - 1, n)])
    # rescale: two outputs overlapping by one limb
    o_a = big.view(-1)[0:2 * (L - 1) * n].view(2, L - 1, n)
    o_b = big.view(-1)[(2 * (L - 1) - 1) * n:(4 * (L - 1) - 1) * n].view(2, L - 1, n)
    with pytest.raises(mhe.MheError, match="alias"):
        ch.eng.rescale_batch([x, y], outs=[o_a, o_b])
    # hmult: out[0] over b[1]
    b1 = big[2:4]
    o0 = big.view(-1)[2 * L * n + n:2 * L * n + n + 2 * (L - 1) * n].view(2, L - 1, n)
    with pytest.raises(mhe.MheError, match="another entry"):
        ch.eng.hmult_batch([x, y], [x, b1], key, outs=[o0, ch.eng.empty(2, L - 1, n)])
    # hmult: out[i] over its own a[i] is fine and gives the oracle's words
    a_host = ch.rand(2, L, n)
    own = ch.up(a_host)
    outs = ch.eng.hmult_batch([own], [own], key, outs=[own.view(-1)[:2 * (L - 1) * n].view(2, L - 1, n)])
    assert np.array_equal(ch.down(outs[0]), ch.oc.hmult(a_host, a_host, ch.down(key)))
    # Galois batch: a bad key level is refused before anything is written
    o = ch.eng.empty(2, L, n)
    o.fill_(7)
    elt = mhe.galois_elt_from_step(ch.log_n, 1)
    with pytest.raises(mhe.MheError, match="kswitch_keys"):
        ch.eng.apply_galois_batch([x, y], [elt, elt], [key, key[:, :, :L]], outs=[o, ch.eng.empty(2, L, n)])
    assert bool((o == 7).all())


@pytest.mark.parametrize("log_n", [13, 16])
def test_seal_surface_batches_equal_one_by_one(log_n):
    """The seal:: batched entry points (rotate_vectors, rescale_to_next_inplace_many,
    relinearize_inplace_many, multiply_reduced_error_many) give the words and scales of the
    one-by-one calls they replace, over mixed levels, shared inputs, NAF-composed and zero steps
    (tests/cpp/seal_batch_test.cpp)."""
    import os
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.check_call(["make", "-s", "-C", os.path.join(root, "fhe-gpt-2_amd", "seal"), "../../build/seal_batch_test"])
    r = subprocess.run([os.path.join(root, "build", "seal_batch_test"), str(log_n)], capture_output=True, text=True,
                       timeout=300)
    print(r.stdout, r.stderr)
    assert r.returncode == 0 and "ALL PASSED" in r.stdout, r.stdout + r.stderr
