"""Pack the reference's pretrained ResNet-20 CIFAR-10 parameters (pretrained_parameters/resnet20_new/*.txt,
read as plain text: no reference code is run) into tests/golden/resnet/resnet20_params.bin: float64
little-endian values concatenated in the order cnn/infer_seal.cpp:3-100 (import_parameters_cifar10)
reads them -- conv weights (conv1, then layer{j}_{k}_conv1/2), batch-norm (bias, running_mean,
running_var, weight) of bn1 then layer{j}_{k}_bn1/bn2, linear weight (100 x 64) and bias (100)."""
import os
import sys

import numpy as np

SRC = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/pretrained_parameters/resnet20_new"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "resnet", "resnet20_params.bin")
END = 2  # ResNet-20: k = 0..2 per stage


def read(name, count):
    v = np.loadtxt(os.path.join(SRC, name), dtype=np.float64).reshape(-1)
    assert v.size >= count, (name, v.size, count)
    return v[:count]


chunks = []
chunks.append(read("conv1_weight.txt", 9 * 3 * 16))
for j in (1, 2, 3):
    for k in range(END + 1):
        co = {1: 16, 2: 32, 3: 64}[j]
        if j == 1 or (j == 2 and k == 0):
            ci = 16
        elif (j == 2 and k != 0) or (j == 3 and k == 0):
            ci = 32
        else:
            ci = 64
        chunks.append(read(f"layer{j}_{k}_conv1_weight.txt", 9 * ci * co))
        chunks.append(read(f"layer{j}_{k}_conv2_weight.txt", 9 * co * co))
chunks += [read(f"bn1_{p}.txt", 16) for p in ("bias", "running_mean", "running_var", "weight")]
for j in (1, 2, 3):
    ci = {1: 16, 2: 32, 3: 64}[j]
    for k in range(END + 1):
        for b in ("bn1", "bn2"):
            chunks += [read(f"layer{j}_{k}_{b}_{p}.txt", ci) for p in ("bias", "running_mean", "running_var", "weight")]
chunks.append(read("linear_weight.txt", 10 * 64))
chunks.append(read("linear_bias.txt", 10))
data = np.concatenate(chunks).astype("<f8")
os.makedirs(os.path.dirname(OUT), exist_ok=True)
data.tofile(OUT)
print(OUT, data.size, "values")
