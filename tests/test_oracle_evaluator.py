"""The checker's own restatement of the modified SEAL evaluator (oracle/evaluator.py, test
infrastructure) on the CPU: the reduced-error ops of SEAL/evaluator.cpp:312-486 in both level
orders and at equal levels, on oracle-encrypted messages, decrypt to the expected values with the
reference's scale bookkeeping (the GPU surface is compared with this restatement word for word in
tests/test_trace_parity.py)."""
import numpy as np
import pytest

import oracle as O
from evaluator import Evaluator, OCt

BITS = [51, 46, 46, 46, 46, 51]  # 5 data primes + special
SCALE = 2.0 ** 40


@pytest.fixture(scope="module")
def env():
    log_n = 12
    n = 1 << log_n
    moduli = O.coeff_modulus_create(n, BITS)
    ctx = O.Context(log_n, moduli)
    K = len(moduli)
    sk = ctx.keygen_secret([1, 2, 3, 4, 5, 6, 7, 8], 0)
    s2 = ctx.dyadic(sk, sk)
    rlk = ctx.kswitch_key([9, 9, 9, 9, 9, 9, 9, 9], sk, s2)
    ev = Evaluator(ctx, K - 1, rlk)
    rng = np.random.default_rng(3)
    return ctx, ev, sk, s2, rng


def encrypt(env, values, L, seed):
    ctx, ev, sk, _, _ = env
    c = ctx.encrypt_zero_symmetric([seed] * 8, sk, L)
    pt = ctx.encode(values, SCALE, L)
    c[0] = ctx.add(c[0], pt)
    return OCt(c, SCALE)


def decrypt(env, c):
    ctx, _, sk, s2, _ = env
    L = c.L
    m = ctx.add(c.data[0], ctx.dyadic(c.data[1], sk[:L]))
    if c.size == 3:
        m = ctx.add(m, ctx.dyadic(c.data[2], s2[:L]))
    return ctx.decode(m, c.scale).real


@pytest.mark.parametrize("op", ["add", "sub", "mul"])
@pytest.mark.parametrize("levels", [(3, 5), (5, 3), (4, 4)])
def test_reduced_error_ops_decrypt(env, op, levels):
    ctx, ev, *_ = env
    rng = env[4]
    n2 = ctx.n // 2
    x, y = rng.uniform(-1, 1, n2), rng.uniform(-1, 1, n2)
    a, b = encrypt(env, x, levels[0], 11), encrypt(env, y, levels[1], 12)
    fn = {"add": ev.add_inplace_reduced_error, "sub": ev.sub_inplace_reduced_error,
          "mul": ev.multiply_inplace_reduced_error}[op]
    fn(a, b)
    assert a.L == min(levels) and a.size == 2
    want = {"add": x + y, "sub": x - y, "mul": x * y}[op]
    got = decrypt(env, a)
    assert np.max(np.abs(got - want)) < 1e-3
    if levels[0] == levels[1]:
        assert a.scale == (b.scale * b.scale if op == "mul" else b.scale)
    elif levels[0] < levels[1]:
        # a keeps the adjusted operand's scale: (a.scale * q_top) / q_top, q_top = b's last prime
        q = float(ctx.moduli[levels[1] - 1])
        adj = SCALE * q / q
        assert a.scale == (adj * adj if op == "mul" else adj)


def test_scale_out_of_bounds_is_raised(env):
    ctx, ev, *_ = env
    a = encrypt(env, np.zeros(ctx.n // 2), 2, 5)
    a.scale = 2.0 ** 60
    with pytest.raises(ValueError, match="scale out of bounds"):
        ev.multiply_inplace(a, a.copy())
