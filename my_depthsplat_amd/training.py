"""Data-parallel training step over the rasterizer (BASELINE configs[3]).

The reference trains per scene with Lightning DDP (`Trainer(num_nodes=...)`, src/main.py:
140-157): each rank encodes and renders its own scenes, the only collective is the gradient
all-reduce of the trainable parameters, then gradient clipping (0.5, config/main.yaml:92) and
AdamW (model_wrapper.py:1104-1158). This module is that step, MI355X-first:

  head (trainable)  -> gaussians_from_head (fused HIP adapter + encoder glue)
                    -> DecoderSplattingCUDA (batched HIP rasterizer, forward + backward)
                    -> fused L1 + MSE loss                     (dls_l1_mse_psnr)
  backward          -> ONE flat fp32 all-reduce of every head gradient (parallel.allreduce_gradients;
                       RCCL over xGMI with the "nccl" backend) -> clip 0.5 -> AdamW.

The dense network in front of the adapter (PromptDA / DINOv2 / DPT; frozen in this fork,
promptda.py:66-73) is out of scope. `GaussianHead` stands in for the trainable Gaussian
regressor + head (encoder_depthsplat.py:96-122) with the vitb head's parameter count
(0.77 M at d_out = 37: a 3.1 MB gradient bucket), so the all-reduce moves what the
reference's would.
The renderer and the loss are arguments, so tests can swap the HIP rasterizer for a dense
torch one (tests/test_parallel.py).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable

import torch
import torch.nn.functional as F
from torch import nn

from .parallel import allreduce_gradients, shard


class _HeadRows(torch.autograd.Function):
    """x [BV, C r^2, h, w] (contiguous fp32 on the GPU) -> rows [BV, (h r)(w r), C] through
    dga_head_rows (one LDS-tiled pass each way; include/dsplat_hip.h)."""

    @staticmethod
    def forward(ctx, x, C: int, r: int):
        from . import _lib
        # the kernel indexes raw pointers by these sizes: a mismatched caller must not reach it
        if x.dim() != 4 or x.dtype != torch.float32 or x.shape[1] != C * r * r:
            raise ValueError(f"head_rows: x must be float32 [BV, C r^2 = {C * r * r}, h, w], got "
                             f"{x.dtype} {tuple(x.shape)}")
        lib = _lib.load()
        _lib.require_gpu(x)
        x = x.contiguous()
        BV, _, h, w = x.shape
        rows = torch.empty((BV, h * r * w * r, C), dtype=torch.float32, device=x.device)
        _lib.check(lib.dga_head_rows(BV, C, r, h, w, x.data_ptr(), rows.data_ptr(), _lib.stream_of(x.device)),
                   "dga_head_rows")
        ctx.dims = (BV, C, r, h, w)
        return rows

    @staticmethod
    def backward(ctx, drows):
        from . import _lib
        BV, C, r, h, w = ctx.dims
        if tuple(drows.shape) != (BV, h * r * w * r, C):
            raise ValueError(f"head_rows backward: gradient {tuple(drows.shape)} != {(BV, h * r * w * r, C)}")
        drows = drows.contiguous().float()
        dx = torch.empty((BV, C * r * r, h, w), dtype=torch.float32, device=drows.device)
        _lib.check(_lib.load().dga_head_rows_bwd(BV, C, r, h, w, drows.data_ptr(), dx.data_ptr(),
                                                 _lib.stream_of(drows.device)), "dga_head_rows_bwd")
        return dx, None, None


def head_rows(x: torch.Tensor, C: int, r: int) -> torch.Tensor:
    """[BV, C r^2, h, w] -> [BV, (h r)(w r), C]: pixel shuffle + "(b v) c h w -> b v (h w) c"
    (encoder_depthsplat.py:224-233 rearranges its head output this way; r = 1 is exactly that).
    GPU tensors: one HIP pass (dga_head_rows); CPU tensors (the gloo tests): the same
    permutation in torch."""
    if x.is_cuda:
        return _HeadRows.apply(x.float(), C, r)
    BV, _, h, w = x.shape
    return x.view(BV, C, r, r, h, w).permute(0, 4, 2, 5, 3, 1).reshape(BV, h * r * w * r, C)


class GaussianHead(nn.Module):
    """Trainable stand-in for the Gaussian regressor + head: context image + depth ->
    per-pixel head channels [B, V, H*W, d_out] (d_out = 1 opacity + 2 offsets + adapter.d_in).
    Works at 1/`down` resolution and pixel-shuffles back to full resolution."""

    def __init__(self, d_out: int, width: int = 108, down: int = 8):
        super().__init__()
        self.down = down
        self.d_out = d_out
        self.stem = nn.Conv2d(4, width, 3, padding=1)
        self.body = nn.Sequential(nn.GELU(), nn.Conv2d(width, 2 * width, 3, padding=1), nn.GELU(),
                                  nn.Conv2d(2 * width, 2 * width, 1), nn.GELU())
        self.out = nn.Conv2d(2 * width, d_out * down * down, 1)
        nn.init.normal_(self.out.weight, std=1e-3)
        nn.init.zeros_(self.out.bias)

    def forward(self, images: torch.Tensor, depths: torch.Tensor) -> torch.Tensor:
        B, V, _, H, W = images.shape
        x = torch.cat([images, depths.reshape(B, V, 1, H, W)], 2).reshape(B * V, 4, H, W)
        x = F.avg_pool2d(x, self.down)
        x = self.out(self.body(self.stem(x)))                   # [BV, d_out r^2, h, w], r = down
        # pixel shuffle + "(b v) c h w -> b v (h w) c" in one pass (head_rows):
        # out[b, v, (hh r + i) W + ww r + j, c] = x[bv, c r^2 + i r + j, hh, ww]
        return head_rows(x, self.d_out, self.down).view(B, V, H * W, self.d_out)


@dataclass
class TrainBatch:
    """One batch of scenes: context images / depths / cameras and target views."""
    images: torch.Tensor       # [B, V, 3, H, W]
    depths: torch.Tensor       # [B, V, H*W, 1, 1]
    ctx_ext: torch.Tensor      # [B, V, 4, 4] c2w
    ctx_k: torch.Tensor        # [B, V, 3, 3] normalised
    tgt_ext: torch.Tensor      # [B, v, 4, 4]
    tgt_k: torch.Tensor        # [B, v, 3, 3]
    near: torch.Tensor         # [B, v]
    far: torch.Tensor          # [B, v]
    target: torch.Tensor       # [B, v, 3, H, W]

    def select(self, idx) -> "TrainBatch":
        idx = list(idx)
        return TrainBatch(*(t[idx] for t in (self.images, self.depths, self.ctx_ext, self.ctx_k, self.tgt_ext,
                                              self.tgt_k, self.near, self.far, self.target)))

    def to(self, device) -> "TrainBatch":
        return TrainBatch(*(t.to(device) for t in (self.images, self.depths, self.ctx_ext, self.ctx_k, self.tgt_ext,
                                                    self.tgt_k, self.near, self.far, self.target)))

    @property
    def n_scenes(self) -> int:
        return self.images.shape[0]


def synthetic_batch(n_scenes: int, n_context: int, n_targets: int, height: int, width: int,
                    seed: int = 0, scene_ids=None) -> TrainBatch:
    """Seeded synthetic scenes (SURVEY §8d cameras; images / depths / targets U-random) on the
    host. Scene i of the global batch depends only on (seed, i), so a rank can build just its
    shard (scene_ids = parallel.shard(n_scenes, rank, world)) and still hold the scenes a
    single process would."""
    from .synthetic import context_cameras, target_cameras
    ids = list(range(n_scenes)) if scene_ids is None else list(scene_ids)
    B, V, v, H, W = len(ids), n_context, n_targets, height, width
    images = torch.empty(B, V, 3, H, W)
    depths = torch.empty(B, V, H * W, 1, 1)
    target = torch.empty(B, v, 3, H, W)
    for k, i in enumerate(ids):
        g = torch.Generator().manual_seed(seed * 100003 + i)
        images[k] = torch.rand(V, 3, H, W, generator=g)
        depths[k] = torch.rand(V, H * W, 1, 1, generator=g) * 9 + 1
        target[k] = torch.rand(v, 3, H, W, generator=g)
    K = torch.tensor([[1.0, 0, 0.5], [0, 1.0, 0.5], [0, 0, 1]])
    ctx = context_cameras(V)[None].repeat(B, 1, 1, 1)
    tgt = target_cameras(context_cameras(V), v)[None].repeat(B, 1, 1, 1)
    return TrainBatch(images, depths, ctx, K.expand(B, V, 3, 3).clone(), tgt, K.expand(B, v, 3, 3).clone(),
                      torch.full((B, v), 0.5), torch.full((B, v), 100.0), target)


def torch_l1_mse(pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    return (pred - target).abs().mean() + (pred - target).square().mean()


class TrainStep:
    """One optimisation step on this rank's scenes. render(gaussians, extrinsics, intrinsics,
    near, far, image_shape) -> colour [B, v, 3, H, W]; loss(pred, target) -> 0-d tensor.

    Optimiser as the reference's (model_wrapper.py:1104-1158 without the monodepth group,
    whose parameters are frozen in this fork): AdamW with lr 2e-4 and weight decay 0.01
    (config/main.yaml:37-41), OneCycleLR over max_steps + 10 steps with pct_start 0.01, cosine
    annealing and no momentum cycling, stepped once per optimisation step; gradient clipping
    0.5 (config/main.yaml:92). max_steps defaults to 150,000 (scripts/re10k_depthsplat_train.sh:9)."""

    def __init__(self, head: GaussianHead, adapter, render: Callable, loss: Callable, lr: float = 2e-4,
                 clip: float = 0.5, world: int = 1, weight_decay: float = 0.01, max_steps: int = 150_000,
                 decoder=None):
        self.head, self.adapter, self.render, self.loss = head, adapter, render, loss
        # decoder (a DecoderSplattingCUDA): adapter + rasterizer as one autograd node
        # (head_render.render_from_head: one fused kernel for the Gaussians' backward); `render`
        # is then unused
        self.decoder = decoder
        self.clip, self.world = clip, world
        self.opt = torch.optim.AdamW(head.parameters(), lr=lr, weight_decay=weight_decay)
        self.sched = torch.optim.lr_scheduler.OneCycleLR(self.opt, lr, max_steps + 10, pct_start=0.01,
                                                         cycle_momentum=False, anneal_strategy="cos")
        self.bucket_bytes = 0

    def forward_backward(self, batch: TrainBatch) -> torch.Tensor:
        from .gaussian_adapter import gaussians_from_head
        H, W = batch.images.shape[-2:]
        raw = self.head(batch.images, batch.depths)
        if self.decoder is not None:
            from .head_render import render_from_head
            color = render_from_head(self.decoder, raw, batch.depths, batch.images, batch.ctx_ext, batch.ctx_k,
                                     self.adapter, batch.tgt_ext, batch.tgt_k, batch.near, batch.far, (H, W))
        else:
            gs = gaussians_from_head(raw, batch.depths, batch.images, batch.ctx_ext, batch.ctx_k, self.adapter)
            color = self.render(gs, batch.tgt_ext, batch.tgt_k, batch.near, batch.far, (H, W))
        loss = self.loss(color, batch.target)
        loss.backward()
        return loss.detach()

    def __call__(self, batch: TrainBatch) -> torch.Tensor:
        loss = self.forward_backward(batch)
        self.bucket_bytes = allreduce_gradients(list(self.head.parameters()), self.world)
        if self.clip:
            torch.nn.utils.clip_grad_norm_(self.head.parameters(), self.clip)
        self.opt.step()
        self.sched.step()
        self.opt.zero_grad(set_to_none=True)
        return loss


def rank_batch(global_batch: TrainBatch, rank: int, world: int) -> TrainBatch:
    """This rank's contiguous shard of the global batch of scenes (parallel.shard)."""
    return global_batch.select(shard(global_batch.n_scenes, rank, world))
