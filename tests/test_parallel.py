"""Multi-process data-parallel helpers on CPU with gloo (world_size 2)."""
from __future__ import annotations

import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from my_depthsplat_amd.parallel import allreduce_gradients, reduce_max, shard


def test_shard_covers_everything():
    for n in (0, 1, 7, 16, 33):
        for w in (1, 2, 3, 8):
            parts = [shard(n, r, w) for r in range(w)]
            assert [i for p in parts for i in p] == list(range(n))
            assert max(len(p) for p in parts) - min(len(p) for p in parts) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(rank)
    lin = torch.nn.Linear(5, 3)
    extra = torch.nn.Parameter(torch.zeros(4))  # no grad on this rank -> contributes zeros
    x = torch.randn(8, 5)
    lin(x).square().sum().backward()
    if rank == 0:
        extra.grad = torch.ones(4)
    before = [p.grad.clone() for p in lin.parameters()]
    nbytes = allreduce_gradients(list(lin.parameters()) + [extra])
    t = reduce_max(float(rank + 1))
    q.put((rank, [b.numpy() for b in before], [p.grad.numpy() for p in lin.parameters()], extra.grad.numpy(),
           nbytes, t))
    dist.barrier()
    dist.destroy_process_group()


def test_allreduce_gradients_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, b0, a0, e0, n0, t0), (_, b1, a1, e1, n1, t1) = res
    for x0, x1, y0, y1 in zip(b0, b1, a0, a1):
        avg = (x0 + x1) / 2
        assert abs(y0 - avg).max() < 1e-6 and abs(y1 - avg).max() < 1e-6
    assert (e0 == 0.5).all() and (e1 == 0.5).all()
    assert n0 == n1 == (15 + 3 + 4) * 4
    assert t0 == t1 == 2.0
