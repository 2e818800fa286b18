"""The exact code path bench.py times, checked word for word against the oracle.

bench.HMultWorkload is the bench's own workload object (not a copy of it): N=2^16, the C2 chain
(44 data limbs + the special prime), L = 44, 32 independent HMults per step issued as 4
mhe_hmult_batch calls of 8 entries (the relin key stream shared through the XCD-grouped entries of
k_ks_row_mac), the prepared key format (residues as doubles), the calls dealt round robin over 4 HIP streams.
One step runs as the bench runs it; every one of the 32 outputs must equal the oracle's HMult
(SEAL/evaluator.cpp:673-814 multiply, :2281-2525 relinearize, util/rns.cpp:737-808 rescale) on the
same inputs and the SEAL-layout key."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("key_format", ["prepared", "seal"])
def test_bench_timed_path_vs_oracle(key_format):
    import torch

    sys.path.insert(0, ROOT)
    import bench
    import oracle as O

    dev = torch.device("cuda", 0)
    w = bench.HMultWorkload(dev, rank=0, limbs=44, batch=32, group=8, streams=4, key_format=key_format,
                            keep_host=True)
    assert [c[1] for c in w.call_streams()] == [8, 8, 8, 8] and sorted({c[2] for c in w.call_streams()}) == [0, 1, 2, 3]
    if key_format == "prepared":
        assert w.eng.key_is_prepared(w.key)
    w.step()
    torch.cuda.synchronize(dev)
    got = w.host(w.out)
    oc = O.Context(bench.LOG_N, w.moduli)
    want, _ = oc.hmult_batch(np.ascontiguousarray(w.host(w.a)), np.ascontiguousarray(w.host(w.b)), w.key_host,
                             threads=min(16, os.cpu_count() or 1))
    bad = [i for i in range(w.B) if not np.array_equal(got[i], want[i])]
    assert not bad, f"HMult entries {bad} differ from the oracle"
    # a second step over the same buffers gives the same words (no state carried between steps)
    w.step()
    torch.cuda.synchronize(dev)
    assert np.array_equal(w.host(w.out), got)
    # and the bench's own rank-0 check passes on these outputs
    res = bench.check_timed_outputs(w, [0, 11, 19, 30], 4)
    assert res["entries"] == [0, 11, 19, 30] and len(res["calls_streams"]) == 4
