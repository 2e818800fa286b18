"""N>1 plumbing of bench.py on CPU: two ranks over gloo.  The relin key drawn on rank 0 reaches
every rank bit-identically (bench.broadcast_key, RCCL on the GPU box), and the job time is
the max over ranks (bench.max_over_ranks)."""
import os
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import bench

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        key = torch.zeros(3, 2, 4, 64, dtype=torch.int64)
        if rank == 0:
            g = torch.Generator().manual_seed(7)
            key.copy_(torch.randint(0, 2**62, key.shape, generator=g))
        bench.broadcast_key(key, src=0)
        t = bench.max_over_ranks(1.0 + rank, torch.device("cpu"))
        q.put((rank, int(key.sum().item()), int(key[2, 1, 3, 63].item()), t))
    finally:
        dist.destroy_process_group()


def test_key_broadcast_and_max_time_gloo_world2():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(2))
    assert res[0][1:3] == res[1][1:3] and res[0][1] != 0   # identical keys on both ranks
    assert res[0][3] == res[1][3] == 2.0                    # max over ranks


# ----------------------------------------------------------------------------- key sharing (§8(e))
def seal_kswitch_stream(parms_id, keys, n):
    """A KSwitchKeys stream in SEAL 3.6's byte format (kswitchkeys.cpp:42-140; serialization.h:60-120):
    header | parms_id | u64 dim1 | per index: u64 dim2 | dim2 PublicKey records (Ciphertext
    save_members: header | parms_id | u8 ntt | u64 size | u64 n | u64 limbs | f64 scale | DynArray).
    keys: {index: array [digits][2][limbs][n]} (a level-truncated key has digits + 1 limbs)."""
    import struct

    def header(size):
        return struct.pack("<HBBBBHQ", 0xA15E, 16, 3, 6, 0, 0, size)

    def dynarray(words):
        return header(16 + 8 + 8 * words.size) + struct.pack("<Q", words.size) + words.astype("<u8").tobytes()

    body = b""
    dim1 = max(keys) + 1
    for i in range(dim1):
        if i not in keys:
            body += struct.pack("<Q", 0)
            continue
        k = keys[i]
        body += struct.pack("<Q", k.shape[0])
        for d in range(k.shape[0]):
            rec = struct.pack("<4Q", *parms_id) + struct.pack("<B", 1) + struct.pack("<3Q", 2, n, k.shape[2]) \
                + struct.pack("<d", 1.0) + dynarray(k[d].reshape(-1))
            body += header(16 + len(rec)) + rec
    payload = struct.pack("<4Q", *parms_id) + struct.pack("<Q", dim1) + body
    return header(16 + len(payload)) + payload


def parse_kswitch_stream(b, n):
    """Independent reader of the same format -> {index: array [digits][2][limbs][n]}."""
    import struct

    import numpy as np

    off = 16
    off += 32
    (dim1,) = struct.unpack_from("<Q", b, off)
    off += 8
    out = {}
    for i in range(dim1):
        (digits,) = struct.unpack_from("<Q", b, off)
        off += 8
        recs = []
        for _ in range(digits):
            off += 16 + 32
            ntt, size, deg, limbs = struct.unpack_from("<B3Q", b, off)
            off += 1 + 24 + 8
            assert (ntt, size, deg) == (1, 2, n)
            off += 16
            (words,) = struct.unpack_from("<Q", b, off)
            off += 8
            recs.append(np.frombuffer(b, dtype="<u8", count=words, offset=off).reshape(2, limbs, n))
            off += 8 * words
        if digits:
            out[i] = np.stack(recs)
    return out


def _share_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, os.path.join(ROOT, "fhe-gpt-2_amd"))
    import hashlib

    import numpy as np

    from mhe import resnet as R

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, parms_id = 64, [11, 22, 33, 44]
        blobs, bufs = [], []
        if rank == 0:
            # the key set of a ResNet runner, as rank 0 would export it: a full relinearization key and
            # level-truncated Galois keys, serialized in SEAL's format, one buffer per key
            rng = np.random.default_rng(5)
            sets = [{0: rng.integers(0, 2**50, size=(3, 2, 4, n), dtype=np.uint64)},
                    {1: rng.integers(0, 2**50, size=(2, 2, 3, n), dtype=np.uint64),
                     4: rng.integers(0, 2**50, size=(1, 2, 2, n), dtype=np.uint64)}]
            for kind, ks in zip((2, 3), sets):
                raw = seal_kswitch_stream(parms_id, ks, n)
                raw += bytes(-len(raw) % 8)
                bufs.append(np.frombuffer(raw, dtype=np.int64).copy())
                blobs.append((kind, 0, 0, bufs[-1].size))

        class Source:
            def key_blobs(self):
                return blobs

        got, done = [], []
        nbuf, nbytes = R.share_keys(
            dist, Source(), torch.device("cpu"), src=0,
            export=lambda i, t: t.copy_(torch.from_numpy(bufs[i])),
            import_=lambda b, t: got.append(t.numpy().tobytes()),
            finish=lambda: done.append(True))
        if rank == 0:
            got = [b.tobytes() for b in bufs]
        parsed = [parse_kswitch_stream(raw, n) for raw in got]
        digest = hashlib.sha256(b"".join(got)).hexdigest()
        # each rank's (decrypted) result reaches rank 0 once, at the end
        results = [None] * world
        dist.all_gather_object(results, {"rank": rank, "logits": [float(rank)] * 10})
        q.put((rank, nbuf, nbytes, digest, {k: v.shape for p in parsed for k, v in p.items()}, bool(done),
               [r["rank"] for r in results]))
    finally:
        dist.destroy_process_group()


def test_key_sharing_serialized_keys_gloo_world2():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_share_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(2))
    r0, r1 = res
    assert r0[1] == r1[1] == 2 and r0[2] == r1[2] > 0          # both buffers moved
    assert r0[3] == r1[3]                                        # bit-identical key streams
    assert r0[4] == r1[4] == {0: (3, 2, 4, 64), 1: (2, 2, 3, 64), 4: (1, 2, 2, 64)}
    assert r1[5] and not r0[5]                                   # the receiver finished its import
    assert r0[6] == r1[6] == [0, 1]                              # results gathered from every rank


# ----------------------------------------------------------------------------- bench.py --gpus N
def _bench_env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    return env


@pytest.mark.parametrize("n", [2, 3])
def test_bench_launcher_spawns_n_ranks(n):
    """`python bench.py --gpus N` without a launcher starts N ranks itself (the driver's command shape
    for the scaling run); --stub runs the rank plumbing on gloo: every rank checks WORLD_SIZE against
    --gpus and joins an all-reduce, and rank 0 reports the world it saw."""
    import json
    import subprocess

    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--stub"], env=_bench_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["ranks_seen"] == n and out["backend"] == "gloo"
    assert out["rank_sum"] == sum(1.0 + k for k in range(n))


def test_bench_rejects_world_mismatch():
    """A launcher-provided WORLD_SIZE that disagrees with --gpus is an error, not a silent 1-rank run."""
    import subprocess

    env = dict(_bench_env(), WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--stub"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in r.stderr
