"""`diff_gaussian_rasterization`-compatible module API on MI355X.

The reference imports `GaussianRasterizationSettings` and `GaussianRasterizer` from the
external CUDA package at src/model/decoder/cuda_splatting.py:5-8 and calls them at
:98-123. This module provides the same names, fields and call contract (the 2-output
API pinned by `image, radii = rasterizer(...)` at :116), so
`from my_depthsplat_amd.rasterizer import GaussianRasterizationSettings, GaussianRasterizer`
is a drop-in. Rendering runs in libdsplat_hip.so; there is no CPU fallback.
"""
from __future__ import annotations

from typing import NamedTuple

import torch
from torch import nn

from . import raster


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool


def _quat_wxyz_to_rot(q: torch.Tensor) -> torch.Tensor:
    # upstream computeCov3D convention: q = (r, x, y, z), used as given (no normalisation)
    r, x, y, z = q.unbind(-1)
    return torch.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
        2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
        2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y),
    ], dim=-1).reshape(q.shape[:-1] + (3, 3))


def cov6_from_scale_rotation(scales: torch.Tensor, rotations: torch.Tensor, modifier: float) -> torch.Tensor:
    """Sigma = R S S^T R^T with S = diag(modifier * scale); returned as (xx,xy,xz,yy,yz,zz)."""
    R = _quat_wxyz_to_rot(rotations)
    M = R * (modifier * scales).unsqueeze(-2)
    sigma = M @ M.transpose(-1, -2)
    return torch.stack([sigma[..., 0, 0], sigma[..., 0, 1], sigma[..., 0, 2], sigma[..., 1, 1],
                        sigma[..., 1, 2], sigma[..., 2, 2]], dim=-1)


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings: GaussianRasterizationSettings):
    s = raster_settings
    P = means3D.shape[0]
    dev = means3D.device
    use_sh = colors_precomp is None
    if cov3Ds_precomp is None:
        cov3Ds_precomp = cov6_from_scale_rotation(scales, rotations, s.scale_modifier)
    if use_sh:
        feats = sh.reshape(P, -1, 3)[None]
    else:
        feats = colors_precomp.reshape(P, 3)[None]
    tx = torch.as_tensor(s.tanfovx, dtype=torch.float32, device=dev).reshape(1)
    ty = torch.as_tensor(s.tanfovy, dtype=torch.float32, device=dev).reshape(1)
    cams = raster.pack_cameras(s.viewmatrix[None], s.projmatrix[None], s.campos.reshape(1, 3), tx, ty,
                               s.bg.reshape(1, 3), torch.zeros(1, dtype=torch.int32, device=dev))
    m2d = means2D if (means2D is not None and means2D.requires_grad) else None
    color, radii = raster.rasterize_views(
        means3D[None], feats, opacities.reshape(1, P), cov3Ds_precomp.reshape(1, P, 6), cams, [0],
        use_sh=use_sh, sh_degree=int(s.sh_degree), image_height=int(s.image_height),
        image_width=int(s.image_width), means2d=m2d)
    return color[0], radii[0]


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings: GaussianRasterizationSettings):
        super().__init__()
        self.raster_settings = raster_settings

    @torch.no_grad()
    def markVisible(self, positions: torch.Tensor) -> torch.Tensor:
        """Frustum test of the upstream API (p_view.z > 0.2)."""
        v = self.raster_settings.viewmatrix
        p_view = positions @ v[:3, :3] + v[3, :3]
        return p_view[:, 2] > 0.2

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None):
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception("Please provide excatly one of either SHs or precomputed colors!")
        if ((scales is None or rotations is None) and cov3D_precomp is None) or (
                (scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!")
        return rasterize_gaussians(means3D, means2D, shs, colors_precomp, opacities, scales, rotations,
                                   cov3D_precomp, self.raster_settings)
