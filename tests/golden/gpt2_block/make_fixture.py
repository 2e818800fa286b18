"""Plain restatement of one GPT-2 transformer block as the encrypted path computes it, and the
fixture the GPU test checks against (tests/golden/gpt2_block/block.bin + block.txt).

The block follows the reference's plain pipeline (plain_approx/full_gpt2.py:94-147: layer_norm ->
attention_layer -> residual -> layer_norm -> mlp -> residual; plain_approx/layers.py:24-116,
plain_approx/attn.py:168-381) with the approximations the encrypted path evaluates in place of the
exact functions:
  * layer norm: row sums by fold + quickSum, mean and variance by 1/d, inverse square root by a
    2nd-order Taylor start at 1 and Newton steps y <- y (1.5 - 0.5 u y^2) (plain_approx/
    iterations.py:15-21; the reference's own start, taylor_expand, has no constant term as written in
    IterApprox.cpp:69-120);
  * softmax: the reference's compute_softmax (PolyApprox.cpp:533-593) on rows of T at stride 2T --
    row max by quickMax of computeMax (Fold.cpp:47-110: 0.5((a-b) sign(0.1(a-b)) + a + b) with the
    composite sign f(f(g(g(x))))), exp(x) ~ (1 + x/64)^64, the causal/padding mask applied
    multiplicatively after exp (attn.py:247's extract mask) and, before the max, masked scores
    pinned to -5 (attn.py:365 adds -1e5, which the sign step of computeMax cannot take), fold + quickSum, Goldschmidt 1/sum
    (IterApprox.cpp:15-68) normalised by 1/T with 8 steps;
  * GELU: the piecewise p / q / x of PolyApprox.cpp:443-504 (plain_approx/poly.py:30-35) with its
    three signs evaluated on alpha (x + shift), alpha = 1/10 so they stay inside [-1, 1], and the last
    piece's indicator s2 + 0.5 (the reference's 0.5 s2 returns +-x/4 there).
Every matrix product is exact here (the encrypted path's placements only move values); softmax is
restated slot by slot because the approximate max depends on the order quickMax combines entries.

Run: python tests/golden/gpt2_block/make_fixture.py  (writes block.bin / block.txt next to itself)
     python tests/golden/gpt2_block/make_fixture.py --full DIR  (GPT-2 dimensions: T 128, d 768,
     12 heads, d_ff 3072, 11 Goldschmidt steps; the ~58 MB of weights are regenerated from the seed
     wherever the test runs, and the committed full/expected.bin -- y and y_exact, with
     full/expected.txt -- pins the result: tests/test_gpt2.py checks a regenerated fixture against it)
"""
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SLOTS = 32768

# block dimensions (reduced GPT-2: 16 tokens, d_model 64, 4 heads of 16, d_ff 256)
T, D, H, F = 16, 64, 4, 256
DH = D // H
SEED = 20261016
GELU_ALPHA = 1.0 / 10.0
NEWTON_ITERS = 3
INV_ITERS = 8
INV_NORM = 1.0 / T
MASKED_SCORE = -5.0   # causal mask: masked scores are replaced by this before the row max

# composite sign (PolyApprox.cpp:103-305, Chebyshev form)
SIGN_F = (-0.6767578125, 1.563049316, -0.02685546875, 0.1384277344, 0.002136230469)
SIGN_G = (-1.121704102, 1.978370667, -0.6178588867, 0.403533935, 0.3557052612)


def cheb(x):
    t2 = 2 * x * x - 1
    t3 = 2 * x * t2 - x
    t4 = 2 * t2 * t2 - 1
    t8 = 2 * t4 * t4 - 1
    return t2, t3, t4, t8


def sign_poly(x, c):
    fq1, fr1, frq2_q, frq2_r, fq3 = c
    t2, t3, t4, t8 = cheb(x)
    return fq1 * x * t2 + fr1 * x + (frq2_q * t3 + frq2_r * x) * t4 + fq3 * x * t8


def sign_function(x):
    # sign_function(2, 2): g, g, then f, f (PolyApprox.cpp:308-334)
    return sign_poly(sign_poly(sign_poly(sign_poly(x, SIGN_G), SIGN_G), SIGN_F), SIGN_F)


def gelu_p(x):
    t2 = 2 * x * x - 1
    return (-0.005337069175 * x - 0.05745879353) * t2 + (-0.4187418723 * x - 0.55528939)


def gelu_q(x):
    t2, _, t4, _ = cheb(x)
    return ((-0.00324699876 * x + 0.1634058825) * t2 + (0.5027208006 * x + 0.1750485092)
            + (0.0001533078376 * x * x + 0.0002609111473 * x - 0.004401064777) * t4)


GELU_REF = False  # --gelu-ref: the x piece weighted by poly.py's 0.5 s2 (GeluLastPiece::reference)


def gelu_block(x):
    y = GELU_ALPHA * x
    s2 = 0.5 * sign_function(y + GELU_ALPHA * -3.0)
    s1 = 0.5 * sign_function(y + GELU_ALPHA * 1.95)
    s0 = 0.5 * sign_function(y + GELU_ALPHA * 4.0)
    b1, b2, b3 = s0 - s1, s1 - s2, (0.5 * s2 if GELU_REF else s2 + 0.5)
    return b1 * gelu_p(x) + b2 * gelu_q(x) + b3 * x


# plain_approx/poly.py:15-28, the power-series gelu_p / gelu_q (coefficients highest power first)
POLY_GELU_P = (-0.010674138350676401, -0.11491758706060971, -0.4134048031372351, -0.49783059647700406)
POLY_GELU_Q = (0.0012264627004247512, 0.0020872891783959252, -0.036434980917200932, -0.0085812866991243648,
               0.36217359096393054, 0.50622871052887408, 0.0072415619838619525)


def _horner(x, coeffs):
    u = np.zeros_like(x)
    for c in coeffs:
        u = u * x + c
    return u


def poly_gelu(x):
    """plain_approx/poly.py:30-35 as written: np.sign of x - 3, x + 1.95, x + 4 (no approximation),
    b1 = s0 - s1, b2 = s1 - s2, b3 = 0.5 s2 (b0 * 0 dropped)."""
    s2, s1, s0 = 0.5 * np.sign(x - 3), 0.5 * np.sign(x + 1.95), 0.5 * np.sign(x + 4)
    return (s0 - s1) * _horner(x, POLY_GELU_P) + (s1 - s2) * _horner(x, POLY_GELU_Q) + 0.5 * s2 * x


def rot(v, k):
    """Evaluator::rotate_vector(v, k): out[i] = v[i + k]."""
    return np.roll(v, -k)


def quick_sum(v, n):
    # Fold.cpp:20-45
    out = v + rot(v, 1)
    acc = 2
    for _ in range(int(math.log2(n)) - 1):
        out = out + rot(out, acc)
        acc *= 2
    return out


def compute_max(a, b):
    # Fold.cpp:47-88
    diff = a - b
    return 0.5 * (diff * sign_function(0.1 * diff) + a + b)


def quick_max(v, n):
    # Fold.cpp:91-110 (bootstrapping is the identity here)
    acc = 1
    for _ in range(int(math.log2(n))):
        v = compute_max(v, rot(v, acc))
        acc *= 2
    return v


def compute_exp(x, r=6):
    y = x / 2.0 ** r + 1.0
    for _ in range(r):
        y = y * y
    return y


def goldschmidt(s, norm, iters):
    # IterApprox.cpp:15-68 with the normalisation as a parameter
    n = np.full_like(s, norm)
    d = norm * s
    for _ in range(iters):
        f = 2.0 - d
        n = n * f
        d = d * f
    return n


def softmax_rows_slots(scores, keep):
    """compute_softmax_rows on one head: scores (T x T) packed at row stride 2T; keep (T x T) 0/1."""
    n = scores.shape[1]
    v = np.zeros(SLOTS)
    km = np.zeros(SLOTS)
    for r in range(scores.shape[0]):
        v[r * 2 * n:r * 2 * n + n] = scores[r]
        km[r * 2 * n:r * 2 * n + n] = keep[r]
    x = v + rot(v, SLOTS - n)
    mx = quick_max(x, n)
    exps = compute_exp(x - mx) * km
    rolled = rot(exps, -n) + exps
    summed = quick_sum(rolled, n)
    out = exps * goldschmidt(summed, INV_NORM, INV_ITERS)
    p = np.stack([out[r * 2 * n:r * 2 * n + n] for r in range(scores.shape[0])])
    return p, {"max_abs_in": float(np.abs(x).max()), "max_row_sum": float(summed.max())}


def layer_norm_block(x, gamma, beta):
    d = x.shape[1]
    mean = x.sum(axis=1, keepdims=True) * (1.0 / d)
    z = x - mean
    u = (z * z).sum(axis=1, keepdims=True) * (1.0 / d)
    t = u - 1.0
    y = (1.0 + (-0.5) * t) + 0.375 * (t * t)
    h = -0.5 * u
    for _ in range(NEWTON_ITERS):
        y = y * ((y * y) * h + 1.5)
    return (z * y) * gamma + beta, u


def block(x, w):
    ranges = {}
    ln1, u1 = layer_norm_block(x, w["ln1_g"], w["ln1_b"])
    q = ln1 @ w["qw"] + w["qb"]
    k = ln1 @ w["kw"] + w["kb"]
    v = ln1 @ w["vw"] + w["vb"]
    keep = np.tril(np.ones((T, T)))
    o = np.zeros((T, D))
    smax_in = 0.0
    for h in range(H):
        sl = slice(h * DH, (h + 1) * DH)
        s = (q[:, sl] @ k[:, sl].T) / math.sqrt(DH)
        s = s * keep + MASKED_SCORE * (1.0 - keep)
        p, info = softmax_rows_slots(s, keep)
        smax_in = max(smax_in, info["max_abs_in"])
        o[:, sl] = p @ v[:, sl]
    attn = o @ w["ow"] + w["ob"]
    x1 = x + attn
    ln2, u2 = layer_norm_block(x1, w["ln2_g"], w["ln2_b"])
    hid = ln2 @ w["fc_w"] + w["fc_b"]
    g = gelu_block(hid)
    f = g @ w["pj_w"] + w["pj_b"]
    y = x1 + f
    y_polygelu = x1 + poly_gelu(hid) @ w["pj_w"] + w["pj_b"]
    ranges.update(var1=(float(u1.min()), float(u1.max())), var2=(float(u2.min()), float(u2.max())),
                  scores=smax_in, hidden=(float(hid.min()), float(hid.max())), x1=float(np.abs(x1).max()),
                  gelu=float(np.abs(g).max()), qkv=float(max(np.abs(q).max(), np.abs(k).max(), np.abs(v).max())))
    return {"ln1": ln1, "q": q, "k": k, "v": v, "attn": attn, "x1": x1, "ln2": ln2, "hidden": hid, "gelu": g,
            "ffn": f, "y": y, "y_polygelu": y_polygelu}, ranges


def exact_block(x, w):
    """The same block with exact layer norm (eps 0), softmax and tanh-GELU (attn.py:388-468,
    test_layers.py:67-94), for the approximation error."""
    def ln(a, g, b):
        m = a.mean(axis=1, keepdims=True)
        var = ((a - m) ** 2).mean(axis=1, keepdims=True)
        return (a - m) / np.sqrt(var) * g + b

    ln1 = ln(x, w["ln1_g"], w["ln1_b"])
    q, k, v = ln1 @ w["qw"] + w["qb"], ln1 @ w["kw"] + w["kb"], ln1 @ w["vw"] + w["vb"]
    o = np.zeros((T, D))
    mask = np.tril(np.ones((T, T)))
    for h in range(H):
        sl = slice(h * DH, (h + 1) * DH)
        s = (q[:, sl] @ k[:, sl].T) / math.sqrt(DH)
        s = np.where(mask == 0, -1e10, s)
        e = np.exp(s - s.max(axis=1, keepdims=True))
        o[:, sl] = (e / e.sum(axis=1, keepdims=True)) @ v[:, sl]
    x1 = x + o @ w["ow"] + w["ob"]
    hid = ln(x1, w["ln2_g"], w["ln2_b"]) @ w["fc_w"] + w["fc_b"]
    g = 0.5 * hid * (1 + np.tanh(math.sqrt(2 / math.pi) * (hid + 0.044715 * hid ** 3)))
    return x1 + g @ w["pj_w"] + w["pj_b"]


# at full width the Q / K weights are drawn at 0.7 / sqrt(d) so that every score stays inside the
# row-max step's domain (computeMax takes sign(0.1 (a - b)), |a - b| <= 10)
FULL = dict(T=128, D=768, H=12, F=3072, INV_ITERS=11, QK_STD=0.7)
QK_STD = 1.0


def set_dims(T_=16, D_=64, H_=4, F_=256, INV_ITERS_=8, QK_STD_=1.0):
    """Block dimensions for the functions above (module globals; the small fixture by default)."""
    global T, D, H, F, DH, INV_ITERS, INV_NORM, QK_STD
    T, D, H, F, INV_ITERS, QK_STD = T_, D_, H_, F_, INV_ITERS_, QK_STD_
    DH = D // H
    INV_NORM = 1.0 / T


def make_inputs(seed=SEED):
    rng = np.random.default_rng(seed)
    x = rng.normal(0.0, 1.0, (T, D))
    w = {
        "ln1_g": 1.0 + 0.1 * rng.normal(size=D), "ln1_b": 0.1 * rng.normal(size=D),
        "qw": rng.normal(0, QK_STD / math.sqrt(D), (D, D)), "qb": 0.05 * rng.normal(size=D),
        "kw": rng.normal(0, QK_STD / math.sqrt(D), (D, D)), "kb": 0.05 * rng.normal(size=D),
        "vw": rng.normal(0, 1.0 / math.sqrt(D), (D, D)), "vb": 0.05 * rng.normal(size=D),
        "ow": rng.normal(0, 0.5 / math.sqrt(D), (D, D)), "ob": 0.05 * rng.normal(size=D),
        "ln2_g": 1.0 + 0.1 * rng.normal(size=D), "ln2_b": 0.1 * rng.normal(size=D),
        "fc_w": rng.normal(0, 0.8 / math.sqrt(D), (D, F)), "fc_b": 0.05 * rng.normal(size=F),
        "pj_w": rng.normal(0, 0.5 / math.sqrt(F), (F, D)), "pj_b": 0.05 * rng.normal(size=D),
    }
    return x, w


ORDER_IN = ["x", "ln1_g", "ln1_b", "qw", "qb", "kw", "kb", "vw", "vb", "ow", "ob", "ln2_g", "ln2_b", "fc_w", "fc_b",
            "pj_w", "pj_b"]
ORDER_OUT = ["ln1", "q", "k", "v", "attn", "x1", "ln2", "hidden", "gelu", "ffn", "y", "y_exact", "y_polygelu"]


def arrays(seed=SEED):
    x, w = make_inputs(seed)
    outs, ranges = block(x, w)
    outs["y_exact"] = exact_block(x, w)
    allv = {"x": x, **w, **outs}
    return [(k, np.atleast_2d(np.asarray(allv[k], dtype="<f8"))) for k in ORDER_IN + ORDER_OUT], ranges


def header():
    return (f"# gpt2 block fixture: T {T} d {D} heads {H} d_ff {F} seed {SEED} alpha {GELU_ALPHA} "
            f"newton {NEWTON_ITERS} inv_iters {INV_ITERS}" + (f" qk_std {QK_STD}" if QK_STD != 1.0 else "")
            + (" gelu_ref 1" if GELU_REF else ""))


def write(dst=HERE, names=None):
    items, ranges = arrays()
    if names is not None:
        items = [(k, a) for k, a in items if k in names]
    off = 0
    lines = [header(), "# name rows cols offset(doubles)"]
    blob = bytearray()
    for name, a in items:
        lines.append(f"{name} {a.shape[0]} {a.shape[1]} {off}")
        blob += a.tobytes()
        off += a.size
    with open(os.path.join(dst, "block.bin"), "wb") as f:
        f.write(bytes(blob))
    with open(os.path.join(dst, "block.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    return ranges


if __name__ == "__main__":
    if "--gelu-ref" in sys.argv:
        sys.argv.remove("--gelu-ref")
        GELU_REF = True
    if len(sys.argv) > 1 and sys.argv[1] in ("--full", "--full-expected"):
        set_dims(*[FULL[k] for k in ("T", "D", "H", "F", "INV_ITERS", "QK_STD")])
        dst = sys.argv[2] if len(sys.argv) > 2 else os.path.join(HERE, "full_ref" if GELU_REF else "full")
        os.makedirs(dst, exist_ok=True)
        if sys.argv[1] == "--full-expected":  # the committed pin: outputs only
            r = write(dst, names={"y", "y_exact", "y_polygelu"} if GELU_REF else {"y", "y_exact"})
            os.replace(os.path.join(dst, "block.bin"), os.path.join(dst, "expected.bin"))
            os.replace(os.path.join(dst, "block.txt"), os.path.join(dst, "expected.txt"))
        else:
            r = write(dst)
        print("ranges:", r)
        sys.exit(0)
    r = write()
    items, _ = arrays()
    d = dict(items)
    print("ranges:", r)
    print("approximate vs exact block: max |y - y_exact| =", float(np.abs(d["y"] - d["y_exact"]).max()))
    sys.exit(0)
