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


@torch.no_grad()
def gather_views(local: torch.Tensor, n_views: int, world: int) -> torch.Tensor:
    """All-gather of per-rank view slices along dim 1 ([b, v_rank, ...] -> [b, n_views, ...] on
    every rank; slices from shard(n_views, r, world), concatenated in rank order). Slices are
    padded to the largest share (one all_gather of equal shapes); a gloo group moves CUDA
    tensors through host memory (rehearsal of the RCCL path)."""
    if world == 1:
        return local
    per = -(-n_views // world)
    pad = local.new_zeros((local.shape[0], per, *local.shape[2:]))
    pad[:, :local.shape[1]] = local
    host = pad.is_cuda and dist.get_backend() == "gloo"
    src = pad.cpu() if host else pad
    parts = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(parts, src)
    out = torch.cat([p[:, :len(shard(n_views, r, world))] for r, p in enumerate(parts)], dim=1)
    return out.to(local.device) if host else out


@torch.no_grad()
def render_view_split(decoder, gaussians, extrinsics, intrinsics, near, far, image_shape, chunk_size,
                      rank: int, world: int, gather: bool = True) -> torch.Tensor:
    """Strong scaling of ONE scene's render (pure rendering, configs B / E): the
    v target views are split over the ranks (parallel.shard, contiguous), the Gaussians are
    replicated read-only on every rank, each rank renders its share in chunks of chunk_size
    (decoder.render_chunked, model_wrapper.py:455-484), then the images are all-gathered
    (gather_views) -> color [b, v, 3, h, w] on every rank. No other exchange."""
    from .decoder import render_chunked
    v = extrinsics.shape[1]
    mine = shard(v, rank, world)
    sl = slice(mine.start, mine.stop)
    local = render_chunked(decoder, gaussians, extrinsics[:, sl], intrinsics[:, sl], near[:, sl], far[:, sl],
                           image_shape, chunk_size).color
    return gather_views(local, v, world) if gather else local
