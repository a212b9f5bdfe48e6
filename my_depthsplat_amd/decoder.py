"""Decoder plugin: drop-in for src/model/decoder/{decoder.py, decoder_splatting_cuda.py,
__init__.py} (Decoder ABC, DecoderOutput, DECODERS registry, get_decoder).

`DecoderSplattingCUDA.forward` keeps the reference signature and outputs
(decoder_splatting_cuda.py:35-67) but renders all B*v views in one batched rasterizer
call over the B scenes' Gaussians: the `repeat(gaussians, "b g ... -> (b v) g ...")`
materialisation of decoder_splatting_cuda.py:53-56 and the per-view loop of
cuda_splatting.py:90-125 are gone.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from dataclasses import dataclass
from typing import Generic, Literal, TypeVar

import torch
from torch import nn

from . import raster
from .cuda_splatting import DepthRenderingMode, render_depth_cuda, render_views


@dataclass
class Gaussians:
    """src/model/types.py:7-12."""
    means: torch.Tensor        # [b, g, 3]
    covariances: torch.Tensor  # [b, g, 3, 3]
    harmonics: torch.Tensor    # [b, g, 3, d_sh]
    opacities: torch.Tensor    # [b, g]


@dataclass
class DecoderOutput:
    """src/model/decoder/decoder.py:19-22."""
    color: torch.Tensor              # [b, v, 3, h, w]
    depth: torch.Tensor | None       # [b, v, h, w]


T = TypeVar("T")


class Decoder(nn.Module, ABC, Generic[T]):
    """src/model/decoder/decoder.py:28-48."""

    def __init__(self, cfg: T, dataset_cfg) -> None:
        super().__init__()
        self.cfg = cfg
        self.dataset_cfg = dataset_cfg

    @abstractmethod
    def forward(self, gaussians: Gaussians, extrinsics: torch.Tensor, intrinsics: torch.Tensor,
                near: torch.Tensor, far: torch.Tensor, image_shape: tuple[int, int],
                depth_mode: DepthRenderingMode | None = None) -> DecoderOutput:
        ...


@dataclass
class DecoderSplattingCUDACfg:
    name: Literal["splatting_cuda"]


def _background(dataset_cfg) -> list[float]:
    if isinstance(dataset_cfg, dict):
        return list(dataset_cfg["background_color"])
    return list(dataset_cfg.background_color)


class DecoderSplattingCUDA(Decoder[DecoderSplattingCUDACfg]):
    """decoder_splatting_cuda.py:19-91 on libdsplat_hip.so. Each decoder owns its rasterizer
    context (`raster_ctx`: binning options and the hints its own calls learn), so decoders of
    different workloads never steer each other's kernels."""

    def __init__(self, cfg: DecoderSplattingCUDACfg, dataset_cfg, **raster_options) -> None:
        super().__init__(cfg, dataset_cfg)
        self.register_buffer("background_color", torch.tensor(_background(dataset_cfg), dtype=torch.float32),
                             persistent=False)
        self.raster_ctx = raster.RasterContext(**raster_options)

    def forward(self, gaussians: Gaussians, extrinsics: torch.Tensor, intrinsics: torch.Tensor,
                near: torch.Tensor, far: torch.Tensor, image_shape: tuple[int, int],
                depth_mode: DepthRenderingMode | None = None) -> DecoderOutput:
        b, v = extrinsics.shape[:2]
        h, w = image_shape
        color = render_views(
            extrinsics.reshape(b * v, 4, 4), intrinsics.reshape(b * v, 3, 3), near.reshape(b * v),
            far.reshape(b * v), image_shape, self.background_color.expand(b * v, 3), gaussians.means,
            gaussians.covariances, gaussians.harmonics, gaussians.opacities,
            view_scene=[i // v for i in range(b * v)], ctx=self.raster_ctx)
        color = color.reshape(b, v, 3, h, w)
        depth = None if depth_mode is None else self.render_depth(
            gaussians, extrinsics, intrinsics, near, far, image_shape, depth_mode)
        return DecoderOutput(color, depth)

    def render_depth(self, gaussians: Gaussians, extrinsics: torch.Tensor, intrinsics: torch.Tensor,
                     near: torch.Tensor, far: torch.Tensor, image_shape: tuple[int, int],
                     mode: DepthRenderingMode = "depth") -> torch.Tensor:
        """decoder_splatting_cuda.py:69-91 (depth colours differ per view, so the
        Gaussians are expanded per view here as in the reference)."""
        b, v = extrinsics.shape[:2]
        rep = lambda t: t[:, None].expand(b, v, *t.shape[1:]).reshape(b * v, *t.shape[1:])  # noqa: E731
        out = render_depth_cuda(extrinsics.reshape(b * v, 4, 4), intrinsics.reshape(b * v, 3, 3),
                                near.reshape(b * v), far.reshape(b * v), image_shape, rep(gaussians.means),
                                rep(gaussians.covariances), rep(gaussians.opacities), mode=mode, ctx=self.raster_ctx)
        return out.reshape(b, v, *image_shape)


def render_chunked(decoder: Decoder, gaussians: Gaussians, extrinsics: torch.Tensor, intrinsics: torch.Tensor,
                   near: torch.Tensor, far: torch.Tensor, image_shape: tuple[int, int],
                   chunk_size: int | None, depth_mode: DepthRenderingMode | None = None) -> DecoderOutput:
    """The test loop's chunked render over target views (model_wrapper.py:455-484): views
    [i*chunk_size, (i+1)*chunk_size) per decoder call, colours concatenated along the view
    axis; the depth (if any) is the first chunk's, as in the reference ("ignore depth").
    chunk_size None renders all views in one call (model_wrapper.py:486-494).

    The colours land in one preallocated [b, v, 3, h, w] buffer (no growing torch.cat), and
    every chunk is one batched decoder call, so a chunk of 10 views of a 5.9 M-Gaussian scene
    is one launch sequence with its key buffers sized for 10 views, not 100."""
    if chunk_size is None:
        return decoder(gaussians, extrinsics, intrinsics, near, far, image_shape, depth_mode=depth_mode)
    if chunk_size <= 0:
        raise ValueError("render_chunk_size must be positive")
    b, v = extrinsics.shape[:2]
    h, w = image_shape
    first, color = None, None
    for start in range(0, v, chunk_size):
        sl = slice(start, min(v, start + chunk_size))
        out = decoder(gaussians, extrinsics[:, sl], intrinsics[:, sl], near[:, sl], far[:, sl], image_shape,
                      depth_mode=depth_mode if first is None else None)
        if first is None:
            first = out
            color = out.color.new_empty((b, v, 3, h, w))
        color[:, sl] = out.color
    return DecoderOutput(color, first.depth)


DECODERS = {"splatting_cuda": DecoderSplattingCUDA}
DecoderCfg = DecoderSplattingCUDACfg


def get_decoder(decoder_cfg: DecoderCfg, dataset_cfg) -> Decoder:
    """src/model/decoder/__init__.py:12-13."""
    return DECODERS[decoder_cfg.name](decoder_cfg, dataset_cfg)
