"""GELU piece fixture: the reference's plain GELU (plain_approx/poly.py:21-35, read as text and restated
here in numpy) and the block's corrected GELU (make_fixture.gelu_block) on the same inputs.

poly.py's gelu takes three half-signs of x - 3, x + 1.95, x + 4 (np.sign), weights its pieces
b1 = s0 - s1 (gelu_p), b2 = s1 - s2 (gelu_q) and b3 = 0.5 s2 (x) -- so x / 4 is added above 3 and
-x / 4 everywhere below it, as written.  The encrypted compute_gelu_block with GeluLastPiece::reference evaluates that
formula with the composite sign of alpha (x + shift) (alpha = 1/10, inside the sign approximation's
[-1, 1]); on inputs at least 0.5 from each breakpoint the composite sign equals np.sign to 1e-10, so
the two must agree within the test's 1e-3.  gelu_p / gelu_q are poly.py's power-series forms (the
same polynomials as PolyApprox.cpp:336-433's Chebyshev forms).

Run: python tests/golden/gpt2_block/make_gelu_ref.py  (writes gelu_ref.bin / gelu_ref.txt next to itself)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_fixture as MF  # noqa: E402

SEED = 20261017
COUNT = 4096
BREAKS = (3.0, -1.95, -4.0)
MARGIN = 0.5


def horner(x, coeffs):
    """coeffs from the highest power down (poly.py's `u = u * x + c` chains)."""
    u = np.zeros_like(x)
    for c in coeffs:
        u = u * x + c
    return u


# poly.py:15-19
POLY_GELU_P = (-0.010674138350676401, -0.11491758706060971, -0.4134048031372351, -0.49783059647700406)
# poly.py:21-28
POLY_GELU_Q = (0.0012264627004247512, 0.0020872891783959252, -0.036434980917200932, -0.0085812866991243648,
               0.36217359096393054, 0.50622871052887408, 0.0072415619838619525)


def poly_gelu(x):
    """plain_approx/poly.py:30-35 as written (b0 * 0 dropped: it is zero)."""
    s2, s1, s0 = 0.5 * np.sign(x - 3), 0.5 * np.sign(x + 1.95), 0.5 * np.sign(x + 4)
    b1, b2, b3 = s0 - s1, s1 - s2, 0.5 * s2
    return b1 * horner(x, POLY_GELU_P) + b2 * horner(x, POLY_GELU_Q) + b3 * x


def inputs(seed=SEED):
    rng = np.random.default_rng(seed)
    x = rng.uniform(-5.5, 5.5, size=4 * COUNT)
    ok = np.ones_like(x, dtype=bool)
    for b in BREAKS:
        ok &= np.abs(x - b) >= MARGIN
    return x[ok][:COUNT]


def arrays():
    x = inputs()
    return [("x", x), ("poly_gelu", poly_gelu(x)), ("gelu_block", MF.gelu_block(x))]


def write(dst=HERE):
    off = 0
    lines = [f"# gelu piece fixture: count {COUNT} seed {SEED} alpha {MF.GELU_ALPHA} margin {MARGIN}",
             "# name rows cols offset(doubles)"]
    blob = bytearray()
    for name, a in arrays():
        a = np.atleast_2d(np.asarray(a, dtype="<f8"))
        lines.append(f"{name} {a.shape[0]} {a.shape[1]} {off}")
        blob += a.tobytes()
        off += a.size
    with open(os.path.join(dst, "gelu_ref.bin"), "wb") as f:
        f.write(bytes(blob))
    with open(os.path.join(dst, "gelu_ref.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    write()
    d = dict(arrays())
    print("max |poly_gelu - gelu_block| =", float(np.abs(d["poly_gelu"] - d["gelu_block"]).max()))
