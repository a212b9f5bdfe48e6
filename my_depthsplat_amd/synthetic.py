"""Seeded synthetic workloads of the reference's shapes.

There is no dataset or checkpoint offline, so scenes are produced the way the reference
produces them at test time — through the Gaussian adapter from a (random) head output:
  cameras   context c2w = identity and +x 0.1 (2 views) or a circle of radius 0.3,
            all looking down +z; targets interpolated between the contexts;
            intrinsics normalised fx = fy = 1, cx = cy = 0.5; near 0.5, far 100, bg 0
  Gaussians images U[0,1], depth U[1,10], raw head ~ N(0,1) -> scales softplus(N-4),
            opacity sigmoid(N), SH DC from the image plus masked N(0,1).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from .decoder import Gaussians
from .gaussian_adapter import GaussianAdapter, GaussianAdapterCfg, gaussians_from_head


@dataclass
class Scene:
    gaussians: Gaussians
    context_images: torch.Tensor      # [B, V, 3, H, W]
    context_extrinsics: torch.Tensor  # [B, V, 4, 4]
    context_intrinsics: torch.Tensor  # [B, V, 3, 3]
    target_extrinsics: torch.Tensor   # [B, v, 4, 4]
    target_intrinsics: torch.Tensor   # [B, v, 3, 3]
    near: torch.Tensor                # [B, v]
    far: torch.Tensor                 # [B, v]
    image_shape: tuple[int, int]


def _c2w(tx: float, ty: float, tz: float, yaw: float = 0.0) -> torch.Tensor:
    m = torch.eye(4)
    c, s = math.cos(yaw), math.sin(yaw)
    m[0, 0], m[0, 2], m[2, 0], m[2, 2] = c, s, -s, c
    m[0, 3], m[1, 3], m[2, 3] = tx, ty, tz
    return m


def context_cameras(n_views: int) -> torch.Tensor:
    if n_views == 2:
        return torch.stack([_c2w(0, 0, 0), _c2w(0.1, 0, 0)])
    poses = []
    for i in range(n_views):
        a = 2 * math.pi * i / n_views
        poses.append(_c2w(0.3 * math.cos(a), 0.3 * math.sin(a), 0.0, yaw=0.05 * math.sin(a)))
    return torch.stack(poses)


def target_cameras(ctx: torch.Tensor, n_targets: int) -> torch.Tensor:
    out = []
    for k in range(n_targets):
        t = (k + 1) / (n_targets + 1)
        i = min(int(t * (ctx.shape[0] - 1)), ctx.shape[0] - 2) if ctx.shape[0] > 1 else 0
        j = min(i + 1, ctx.shape[0] - 1)
        f = t * (ctx.shape[0] - 1) - i
        m = ctx[i].clone()
        m[:3, 3] = (1 - f) * ctx[i, :3, 3] + f * ctx[j, :3, 3]
        out.append(m)
    return torch.stack(out)


def make_scene(batch: int = 1, n_context: int = 2, n_targets: int = 3, height: int = 256, width: int = 256,
               seed: int = 0, device: str | torch.device = "cuda", sh_degree: int = 2) -> Scene:
    g = torch.Generator().manual_seed(seed)
    adapter = GaussianAdapter(GaussianAdapterCfg(1e-10, 3.0, sh_degree))
    B, V, h, w = batch, n_context, height, width
    images = torch.rand(B, V, 3, h, w, generator=g)
    depths = (torch.rand(B, V, h * w, 1, 1, generator=g) * 9 + 1)
    head = torch.randn(B, V, h * w, 3 + adapter.d_in, generator=g)
    ctx = context_cameras(V)[None].repeat(B, 1, 1, 1)
    K = torch.tensor([[1.0, 0, 0.5], [0, 1.0, 0.5], [0, 0, 1]])
    ctx_k = K.expand(B, V, 3, 3).clone()
    tgt = target_cameras(context_cameras(V), n_targets)[None].repeat(B, 1, 1, 1)
    tgt_k = K.expand(B, n_targets, 3, 3).clone()
    dev = torch.device(device)
    to = lambda t: t.to(dev)  # noqa: E731
    adapter = adapter.to(dev)
    with torch.no_grad():
        gs = gaussians_from_head(to(head), to(depths), to(images), to(ctx), to(ctx_k), adapter)
    near = torch.full((B, n_targets), 0.5, device=dev)
    far = torch.full((B, n_targets), 100.0, device=dev)
    return Scene(gs, to(images), to(ctx), to(ctx_k), to(tgt), to(tgt_k), near, far, (h, w))
