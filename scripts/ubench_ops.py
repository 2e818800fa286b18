"""Per-operation timing at ResNet levels (N=2^16, the CNN chain 51 + 16x46 + 14x51 + special 51).

Times the evaluator's small-level building blocks through the C ABI with HIP events on the engine's
stream: rescale (1 and 4 ciphertexts per launch), key switch / relinearize (1 and 4), rotations with
4 distinct keys, forward NTT of one ciphertext, and an HMult.  Prints one JSON line per operation.
Used for A/B runs of library variants (MHE_LIB_PATH=build/var/NAME/libmhe.so).

    python scripts/ubench_ops.py [--limbs 31] [--reps 50]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-gpt-2_amd"))

import torch  # noqa: E402

import mhe  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--limbs", type=int, default=31)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--ops", default="rescale,rescale4,ks,ks4,ks4s,rot4,ntt,hmult")
    ap.add_argument("--bsgs", default="8x7", help="inputs x rotations of the bsgs op (keys shared over inputs)")
    ap.add_argument("--hoist", type=int, default=None, help="hoisted rotations on (1) / off (0); default: the context's")
    a = ap.parse_args()
    log_n, n = 16, 1 << 16
    bits = [51] + [46] * 16 + [51] * 14 + [51]
    moduli = mhe.coeff_modulus_create(n, bits)
    eng = mhe.Engine(log_n, moduli, device=0)
    if a.hoist is not None:
        eng.set_hoist(bool(a.hoist))
    K, L = len(moduli), a.limbs
    qs = torch.tensor(np.array(moduli, np.uint64).view(np.int64), device=eng.torch_device)

    def rnd(*shape, limbs):
        # residues below each limb's prime (shape [..., limbs, n])
        g = torch.randint(0, 2**62, shape, dtype=torch.int64, device=eng.torch_device)
        q = qs[:limbs].view(*([1] * (len(shape) - 2)), limbs, 1)
        return torch.remainder(g, q)

    eng.reserve(K - 1)
    keys = [rnd(L, 2, K, n, limbs=K) for _ in range(4)]
    for k in keys:
        eng.key_prepare(k)
    cts = [rnd(2, L, n, limbs=L) for _ in range(8)]
    ct3 = [rnd(3, L, n, limbs=L) for _ in range(4)]
    outs = [eng.empty(2, L - 1, n) for _ in range(8)]
    rot_out = [eng.empty(2, L, n) for _ in range(4)]
    elts = [pow(5, s, 2 * n) for s in (1, 2, 4, 8)]
    # bsgs: the BSGS baby steps of several images (FiberBatch): each input rotated R ways, the R keys
    # shared by the inputs -- the hoisted path (csrc/hoist.h) when hoisting is on (--hoist 1)
    if "bsgs" in a.ops:
        H, R = (int(x) for x in a.bsgs.split("x"))
        bkeys = [rnd(L, 2, K, n, limbs=K) for _ in range(R)]
        for k in bkeys:
            eng.key_prepare(k)
        bin_ = [rnd(2, L, n, limbs=L) for _ in range(H)]
        b_in = [c for c in bin_ for _ in range(R)]
        b_el = [pow(5, s + 1, 2 * n) for _ in range(H) for s in range(R)]
        b_k = [bkeys[s] for _ in range(H) for s in range(R)]
        b_out = [eng.empty(2, L, n) for _ in b_in]

    ops = {
        "rescale": lambda: eng.rescale_to_next(cts[0], outs[0]),
        "rescale4": lambda: eng.rescale_batch(cts[:4], outs[:4]),
        "rescale8": lambda: eng.rescale_batch(cts, outs),
        "ks": lambda: eng.relinearize(ct3[0], keys[0]),
        "ks4": lambda: eng.switch_key_batch([c[:2] for c in ct3], [c[2] for c in ct3], keys),
        "ks4s": lambda: eng.switch_key_batch([c[:2] for c in ct3], [c[2] for c in ct3], [keys[0]] * 4),
        "rot4": lambda: eng.apply_galois_batch(cts[:4], elts, keys, rot_out),
        "bsgs": lambda: eng.apply_galois_batch(b_in, b_el, b_k, b_out),
        "ntt": lambda: eng.ntt_forward(cts[1]),
        "hmult": lambda: eng.hmult(cts[2], cts[3], keys[0], outs[1]),
        # elementwise, one ciphertext (2 x L limbs): HBM-bound, so us -> GB/s directly
        "add": lambda: eng.add(cts[0], cts[1], rot_out[0]),
        "mulplain": lambda: eng.multiply_plain(cts[0], cts[2][0], rot_out[0]),
    }
    st = torch.cuda.current_stream(eng.torch_device)
    for name in a.ops.split(","):
        f = ops[name]
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record(st)
        for _ in range(a.reps):
            f()
        t1.record(st)
        torch.cuda.synchronize()
        us = t0.elapsed_time(t1) * 1000 / a.reps
        print(json.dumps({"op": name if name != "bsgs" else "bsgs" + a.bsgs, "limbs": L, "us": round(us, 2),
                          "hoist": int(eng.hoist()[0]), "lib": os.environ.get("MHE_LIB_PATH", "libmhe.so")}),
              flush=True)


if __name__ == "__main__":
    main()
