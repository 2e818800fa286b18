"""Debug probe: run each engine op on a buffer followed by a guard region and report any write
past the buffer's end (ResNet chain, N=2^16)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fhe-gpt-2_amd"))
import mhe  # noqa: E402
import torch  # noqa: E402

BITS = [51] + [46] * 16 + [51] * 14 + [51]
n = 1 << 16
moduli = mhe.coeff_modulus_create(n, BITS)
eng = mhe.Engine(16, moduli)
K = len(moduli)
G = 1 << 20  # guard words
PAT = 0x0BADF00D0BADF00D


def guarded(*shape):
    words = int(np.prod(shape))
    buf = torch.zeros(words + G, dtype=torch.int64, device="cuda")
    buf[words:] = PAT
    return buf, buf[:words].view(*shape)


def check(name, buf, words):
    torch.cuda.synchronize()
    g = buf[words:]
    bad = (g != PAT).nonzero()
    if bad.numel():
        print(f"OVERRUN {name}: {bad.numel()} guard words written, first at +{int(bad[0])} last at +{int(bad[-1])}", flush=True)
    else:
        print(f"ok {name}", flush=True)


def fill(t, limbs_dim=-2):
    L = t.shape[limbs_dim]
    for l in range(L):
        idx = [slice(None)] * t.dim()
        idx[limbs_dim] = l
        t[tuple(idx)] = torch.randint(0, moduli[l] - 1, t[tuple(idx)].shape, device="cuda")


for p, l in [(1, 1), (1, 3), (1, 20), (1, 31), (1, 32), (2, 20), (2, 31), (2, 32), (3, 17)]:
    for fn in ("ntt_forward", "ntt_inverse"):
        buf, t = guarded(p, l, n)
        fill(t)
        getattr(eng, fn)(t)
        check(f"{fn} polys={p} limbs={l}", buf, p * l * n)
for kind in ("uniform", "ternary", "normal"):
    for l in (1, 20, 32):
        buf, t = guarded(l, n)
        eng.sample(kind, l, 5, 7, out=t)
        check(f"sample {kind} limbs={l}", buf, l * n)
for l in (3, 20, 32):
    a = eng.empty(1, l, n); fill(a)
    b = eng.empty(l, n); fill(b, 0)
    buf, o = guarded(1, l, n)
    eng.multiply_plain(a, b, out=o)
    check(f"multiply_plain limbs={l}", buf, l * n)
    buf, o = guarded(1, l, n)
    eng.add(a, a, out=o)
    check(f"add limbs={l}", buf, l * n)
    buf, o = guarded(1, l, n)
    eng.multiply_scalar(a, [1] * l, out=o)
    check(f"multiply_scalar limbs={l}", buf, l * n)
    buf, o = guarded(1, l, n)
    eng.permute_galois(a, 5, out=o)
    check(f"permute_galois limbs={l}", buf, l * n)
for L in (3, 20, 31):
    a = eng.empty(2, L, n); fill(a)
    buf, o = guarded(2, L - 1, n)
    eng.rescale_to_next(a, out=o)
    check(f"rescale L={L}", buf, 2 * (L - 1) * n)
    buf, o = guarded(2, L - 1, n)
    eng.mod_switch_drop(a, out=o)
    check(f"mod_switch_drop L={L}", buf, 2 * (L - 1) * n)
    buf, o = guarded(3, L, n)
    eng.square(a, out3=o)
    check(f"square L={L}", buf, 3 * L * n)
    key = eng.empty(L, 2, L + 1, n); fill(key)
    buf, ct = guarded(2, L, n)
    fill(ct)
    eng.apply_galois(ct, 5, key)
    check(f"apply_galois L={L} truncated key", buf, 2 * L * n)
    buf, ct3 = guarded(3, L, n)
    fill(ct3)
    eng.relinearize(ct3, key)
    check(f"relinearize L={L} truncated key", buf, 3 * L * n)
c1 = eng.empty(2, 1, n); fill(c1)
buf, o = guarded(2, 31, n)
eng.modraise(c1, 31, out=o)
check("modraise 31", buf, 2 * 31 * n)
