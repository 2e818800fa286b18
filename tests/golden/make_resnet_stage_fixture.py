"""Extracts the stage sequence of the reference's ResNet-20 run on image 0 -- each logged op with its
remaining level (chain index) and printed scale -- from /root/reference/result/
resnet20_cifar10_image0.txt (written by cnn/infer_seal.cpp:404-577) into
tests/golden/resnet/resnet20_image0_stages.json.  Data only: op names, levels, scales as printed.
Run here once (the reference tree does not exist on the GPU box)."""
import json
import os
import re

SRC = "/root/reference/result/resnet20_cifar10_image0.txt"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "resnet", "resnet20_image0_stages.json")


def parse(text):
    """[(layer, op, level, scale)] from a log in the reference's *_print format."""
    stages, layer, op, level = [], None, None, None
    for line in text.splitlines():
        m = re.match(r"^layer (\d+)$", line)
        if m:
            layer = int(m.group(1))
            continue
        if line.endswith("...") and not line.startswith("("):
            op = line[:-3]
            continue
        m = re.match(r"^remaining level : (\d+)$", line)
        if m:
            level = int(m.group(1))
            continue
        m = re.match(r"^scale: (\S+)$", line)
        if m and op is not None:
            stages.append({"layer": layer, "op": op, "level": level, "scale": m.group(1)})
            op = None
    return stages


if __name__ == "__main__":
    stages = parse(open(SRC).read())
    json.dump({"source": "result/resnet20_cifar10_image0.txt", "stages": stages}, open(OUT, "w"), indent=0)
    print(len(stages), "stages ->", OUT)
