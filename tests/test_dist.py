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
