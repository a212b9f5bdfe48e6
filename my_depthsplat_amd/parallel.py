"""Per-scene data parallelism over one node.

One process per GPU (torchrun), `torch.distributed` with the "nccl" backend (= RCCL on
ROCm, over xGMI). The rasterizer path itself has no exchange: each rank renders its own
scenes (or its own target views of a shared scene). The only collective is the gradient
all-reduce of the trainable parameters in training (1.7 / 3.1 / 4.0 MB fp32 for the
vits / vitb / vitl heads, §5): latency-bound over xGMI, so it is issued as ONE flat
bucket per step rather than per-parameter or per-layer calls.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_rank() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def init_distributed(backend: str | None = None) -> tuple[int, int, int]:
    """Initialise from torchrun env (MASTER_ADDR defaults to 127.0.0.1). Returns
    (rank, local_rank, world). Backend: "nccl" (RCCL) on GPUs, "gloo" on CPU."""
    rank, local, world = env_rank()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, local, world


def shard(n_items: int, rank: int, world: int) -> range:
    """Contiguous, balanced split of n_items (scenes or target views) over ranks."""
    base, extra = divmod(n_items, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


@torch.no_grad()
def allreduce_gradients(params, world: int | None = None) -> int:
    """Average .grad of `params` over all ranks with ONE all-reduce of a flat fp32 bucket.
    Returns the bucket size in bytes. Parameters without a gradient contribute zeros (and
    receive the average), so every rank issues the identical collective."""
    params = [p for p in params if p.requires_grad]
    if not params:
        return 0
    world = dist.get_world_size() if world is None else world
    grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in params]
    flat = torch.cat([g.reshape(-1).float() for g in grads])
    if world > 1:
        if flat.is_cuda and dist.get_backend() == "gloo":  # gloo rehearsal of the GPU path
            host = flat.cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM)
            flat.copy_(host)
        else:
            dist.all_reduce(flat, op=dist.ReduceOp.SUM)
        flat /= world
    off = 0
    for p, g in zip(params, grads):
        n = g.numel()
        upd = flat[off:off + n].view_as(g).to(g.dtype)
        if p.grad is None:
            p.grad = upd.clone()
        else:
            p.grad.copy_(upd)
        off += n
    return flat.numel() * 4


@torch.no_grad()
def reduce_max(value: float, device=None) -> float:
    """Max over ranks (bench timing: the slowest rank defines the job time)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
