"""One key set for several runners: the runner that generated the keys exports
every buffer (secret, public, relinearization, level-truncated Galois keys) as device memory, a
second runner imports them (what each rank does after the RCCL broadcast of mhe.resnet.share_keys)
and both classify the same image.  Same keys and image: the same label, logits equal up to the
encryption noise of two fresh encryptions.  The N>1 transport itself is covered on CPU by
tests/test_dist.py (gloo, world 2)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-gpt-2_amd"))


@pytest.mark.gpu
def test_exported_keys_drive_a_second_runner():
    import torch

    from mhe import resnet as R

    params = os.path.join(ROOT, "tests", "golden", "resnet", "resnet20_params.bin")
    comp = os.path.join(ROOT, "tests", "golden", "comp")
    os.environ["MHE_DEVICE"] = "0"
    a = R.Runner(20, params, comp, generate_keys=True)
    b = R.Runner(20, params, comp, generate_keys=False)
    blobs = a.key_blobs()
    kinds = sorted({k for k, *_ in blobs})
    assert kinds == [0, 1, 2, 3] and sum(1 for k, *_ in blobs if k == 3) == a.info()["galois_keys"]
    moved = 0
    for i, (kind, index, limbs, words) in enumerate(blobs):
        t = torch.empty(words, dtype=torch.int64, device="cuda:0")
        a.export_key(i, t.data_ptr())
        if kind in (2, 3):  # the runner's keys are prepared (mhe_key_prepare); exports are SEAL's layout
            # a prepared word (a double >= 1, or -0.0) is >= 2^61 as u64: negative or >= 2^61 as int64
            assert not bool(((t < 0) | (t >= (1 << 61))).any()), (kind, index)
        b.import_key(kind, index, limbs, words, t.data_ptr())
        moved += words * 8
        del t
    b.finish_import()
    assert b.info()["galois_keys"] == a.info()["galois_keys"]
    assert abs(b.info()["galois_key_gb"] - a.info()["galois_key_gb"]) < 1e-9
    img = np.random.default_rng(3).uniform(-2.5, 2.5, size=(1, 3072))
    ra, rb = a.infer_batch(img, 1), b.infer_batch(img, 1)
    assert ra["labels"][0] == rb["labels"][0]
    assert np.max(np.abs(ra["logits"] - rb["logits"])) < 0.05 * np.max(np.abs(ra["logits"]))
    print(f"moved {moved / 1e9:.1f} GB of keys; logits {ra['logits'][0][:3]} vs {rb['logits'][0][:3]}")
    a.close()
    b.close()
