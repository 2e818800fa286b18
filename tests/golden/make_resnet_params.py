"""Pack the reference's pretrained ResNet CIFAR-10 parameters (pretrained_parameters/resnet<L>_new/*.txt,
read as plain text: no reference code is run) into tests/golden/resnet/, values concatenated in the
order cnn/infer_seal.cpp:3-100 (import_parameters_cifar10) reads them -- conv weights (conv1, then
layer{j}_{k}_conv1/2), batch-norm (bias, running_mean, running_var, weight) of bn1 then
layer{j}_{k}_bn1/bn2, linear weight (10 x 64) and bias (10).

  python make_resnet_params.py [layers=20] [src_dir]

ResNet-20 is written as float64 (resnet20_params.bin).  Larger networks are written losslessly in
the ".d7" format, 4 bytes per value: every value in the reference's files is printed "%e" with 7
significant digits (d.dddddde+XX), so it is exactly m * 10^(x - 6) with |m| < 10^7 < 2^24:
word = sign << 31 | (x + 64) << 24 | m.  The loader turns (m, x) back into the decimal text and
parses it with strtod, which yields the same double as parsing the reference's own text."""
import os
import re
import struct
import sys

import numpy as np

DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "resnet")
TOKEN = re.compile(r"^(-?)([0-9])\.([0-9]{6})e([-+][0-9]{2})$")


def read_text(src, name, count):
    with open(os.path.join(src, name)) as f:
        toks = f.read().split()
    assert len(toks) >= count, (name, len(toks), count)
    return toks[:count]


def tokens(src, layers):
    END = (layers - 2) // 6 - 1  # infer_seal.cpp: end_num (20 -> 2, 110 -> 17)
    out = read_text(src, "conv1_weight.txt", 9 * 3 * 16)
    for j in (1, 2, 3):
        for k in range(END + 1):
            co = {1: 16, 2: 32, 3: 64}[j]
            if j == 1 or (j == 2 and k == 0):
                ci = 16
            elif (j == 2 and k != 0) or (j == 3 and k == 0):
                ci = 32
            else:
                ci = 64
            out += read_text(src, f"layer{j}_{k}_conv1_weight.txt", 9 * ci * co)
            out += read_text(src, f"layer{j}_{k}_conv2_weight.txt", 9 * co * co)
    for p in ("bias", "running_mean", "running_var", "weight"):
        out += read_text(src, f"bn1_{p}.txt", 16)
    for j in (1, 2, 3):
        c = {1: 16, 2: 32, 3: 64}[j]
        for k in range(END + 1):
            for b in ("bn1", "bn2"):
                for p in ("bias", "running_mean", "running_var", "weight"):
                    out += read_text(src, f"layer{j}_{k}_{b}_{p}.txt", c)
    out += read_text(src, "linear_weight.txt", 10 * 64)
    out += read_text(src, "linear_bias.txt", 10)
    return out


def pack_d7(toks):
    words = []
    for t in toks:
        m = TOKEN.match(t)
        assert m, t
        mant = int(m.group(2) + m.group(3))
        x = int(m.group(4))
        assert -64 <= x < 64
        words.append((1 << 31 if m.group(1) else 0) | ((x + 64) << 24) | mant)
    return struct.pack(f"<{len(words)}I", *words)


def unpack_d7(raw):
    """Test-side decoder (same rule as the C++ loader)."""
    w = np.frombuffer(raw, dtype="<u4").tolist()
    return np.array([float(f"{'-' if v >> 31 else ''}{v & 0xFFFFFF}e{((v >> 24) & 0x7F) - 64 - 6}") for v in w])


if __name__ == "__main__":
    LAYERS = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    SRC = sys.argv[2] if len(sys.argv) > 2 else f"/root/reference/pretrained_parameters/resnet{LAYERS}_new"
    toks = tokens(SRC, LAYERS)
    os.makedirs(DIR, exist_ok=True)
    if LAYERS == 20:
        out = os.path.join(DIR, "resnet20_params.bin")
        np.array([float(t) for t in toks], dtype="<f8").tofile(out)
    else:
        out = os.path.join(DIR, f"resnet{LAYERS}_params.d7")
        with open(out, "wb") as f:
            f.write(pack_d7(toks))
    print(out, len(toks), "values")
