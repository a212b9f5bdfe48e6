"""Gaussian adapter: drop-in for src/model/encoder/common/gaussian_adapter.py and
gaussians.py (GaussianAdapterCfg, GaussianAdapter, RGB2SH, quaternion_to_matrix,
build_covariance) plus the encoder glue of encoder_depthsplat.py:258-273.

Same names, config fields, argument meaning and output shapes as the reference. On the
device, `GaussianAdapter.forward` runs the fused HIP kernel (dga_adapter_forward/backward:
one launch per direction; adapter_hip.py) and `gaussians_from_head` the same kernel with the
encoder glue fused in (dga_adapter_fwd/bwd). The torch composition below is what host
tensors run: the fp32 reference the kernels are tested against (tests/test_adapter_gpu.py)
and the synthetic-data builder for the CPU oracle. It is pinned by tests/golden/adapter.npz,
recorded from the reference modules (identity rotations: e3nn is absent offline).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn.functional as F
from torch import nn

from .projection import get_world_rays, sample_image_grid
from .sh_rotation import rotate_sh

SH_C0 = 0.28209479177387814


def RGB2SH(rgb: torch.Tensor) -> torch.Tensor:  # noqa: N802 (reference name)
    """gaussian_adapter.py:126-128."""
    return (rgb - 0.5) / SH_C0


def quaternion_to_matrix(quaternions: torch.Tensor, eps: float = 1e-8) -> torch.Tensor:
    """Scipy-order (x, y, z, w) quaternion -> rotation (gaussians.py:8-30)."""
    i, j, k, r = quaternions.unbind(-1)
    two_s = 2 / ((quaternions * quaternions).sum(dim=-1) + eps)
    rows = (
        1 - two_s * (j * j + k * k), two_s * (i * j - k * r), two_s * (i * k + j * r),
        two_s * (i * j + k * r), 1 - two_s * (i * i + k * k), two_s * (j * k - i * r),
        two_s * (i * k - j * r), two_s * (j * k + i * r), 1 - two_s * (i * i + j * j),
    )
    return torch.stack(rows, dim=-1).reshape(quaternions.shape[:-1] + (3, 3))


def build_covariance(scale: torch.Tensor, rotation_xyzw: torch.Tensor) -> torch.Tensor:
    """R S S^T R^T (gaussians.py:33-44)."""
    S = scale.diag_embed()
    R = quaternion_to_matrix(rotation_xyzw)
    return R @ S @ S.transpose(-1, -2) @ R.transpose(-1, -2)


@dataclass
class GaussianAdapterCfg:
    gaussian_scale_min: float
    gaussian_scale_max: float
    sh_degree: int


@dataclass
class AdapterGaussians:
    """gaussian_adapter.py:14-21 (the adapter's own, richer, Gaussians)."""
    means: torch.Tensor
    covariances: torch.Tensor
    scales: torch.Tensor
    rotations: torch.Tensor
    harmonics: torch.Tensor
    opacities: torch.Tensor


class GaussianAdapter(nn.Module):
    """gaussian_adapter.py:31-123."""

    def __init__(self, cfg: GaussianAdapterCfg):
        super().__init__()
        self.cfg = cfg
        mask = torch.ones((self.d_sh,), dtype=torch.float32)
        for degree in range(1, cfg.sh_degree + 1):
            mask[degree ** 2:(degree + 1) ** 2] = 0.1 * 0.25 ** degree
        self.register_buffer("sh_mask", mask, persistent=False)

    @property
    def d_sh(self) -> int:
        return (self.cfg.sh_degree + 1) ** 2

    @property
    def d_in(self) -> int:
        return 7 + 3 * self.d_sh

    def forward(self, extrinsics, intrinsics, coordinates, depths, opacities, raw_gaussians, image_shape,
                eps: float = 1e-8, point_cloud=None, input_images=None) -> AdapterGaussians:
        # The fused HIP kernel differentiates w.r.t. raw_gaussians, coordinates and depths; the
        # reference's autograd also reaches extrinsics, intrinsics and input_images. A caller
        # that optimises those (pose refinement) gets the torch composition on the device, so
        # its gradients are never silently dropped.
        cam_grad = any(t is not None and t.requires_grad for t in (extrinsics, intrinsics, input_images))
        if raw_gaussians.is_cuda and not (cam_grad and torch.is_grad_enabled()):
            from .adapter_hip import adapter_forward_hip
            return adapter_forward_hip(self, extrinsics, intrinsics, coordinates, depths, opacities, raw_gaussians,
                                       image_shape, eps, input_images)
        return self.forward_torch(extrinsics, intrinsics, coordinates, depths, opacities, raw_gaussians,
                                  image_shape, eps, point_cloud, input_images)

    def forward_torch(self, extrinsics, intrinsics, coordinates, depths, opacities, raw_gaussians, image_shape,
                      eps: float = 1e-8, point_cloud=None, input_images=None) -> AdapterGaussians:
        """The reference's torch composition (host tensors; the kernels' fp32 reference)."""
        scales, rotations, sh = raw_gaussians.split((3, 4, 3 * self.d_sh), dim=-1)
        scales = torch.clamp(F.softplus(scales - 4.0), min=self.cfg.gaussian_scale_min,
                             max=self.cfg.gaussian_scale_max)
        if input_images is None:
            raise ValueError("GaussianAdapter.forward needs input_images (gaussian_adapter.py:69)")
        rotations = rotations / (rotations.norm(dim=-1, keepdim=True) + eps)
        sh = sh.unflatten(-1, (3, self.d_sh))
        sh = sh.broadcast_to((*opacities.shape, 3, self.d_sh)) * self.sh_mask
        b, v, c, h, w = input_images.shape
        imgs = input_images.permute(0, 1, 3, 4, 2).reshape(b, v, h * w, 1, 1, c)
        sh = sh.clone()
        sh[..., 0] = sh[..., 0] + RGB2SH(imgs)
        cov = build_covariance(scales, rotations)
        c2w = extrinsics[..., :3, :3]
        cov = c2w @ cov @ c2w.transpose(-1, -2)
        origins, directions = get_world_rays(coordinates, extrinsics, intrinsics)
        means = origins + directions * depths[..., None]
        return AdapterGaussians(
            means=means, covariances=cov, harmonics=rotate_sh(sh, c2w[..., None, :, :]), opacities=opacities,
            scales=scales, rotations=rotations.broadcast_to((*scales.shape[:-1], 4)))


def gaussians_from_head(head: torch.Tensor, depths: torch.Tensor, images: torch.Tensor, extrinsics: torch.Tensor,
                        intrinsics: torch.Tensor, adapter: GaussianAdapter):
    """Encoder glue (encoder_depthsplat.py:224-346) for one surface / one Gaussian per pixel:
    head [B, V, H*W, C] raw head channels (C = 1 + 2 + adapter.d_in: opacity logit, pixel
    offset logits, adapter input), depths [B, V, H*W, 1, 1], images [B, V, 3, H, W],
    extrinsics [B, V, 4, 4] (c2w), intrinsics [B, V, 3, 3] (normalised).
    Returns the decoder's Gaussians (means [B, G, 3], covariances [B, G, 3, 3],
    harmonics [B, G, 3, d_sh], opacities [B, G]) with G = V*H*W, view-major.

    Device tensors go through the fused HIP adapter (dga_adapter_fwd/bwd: one pass, grads
    for head and depths; the images get none). Host tensors (synthetic-data generation for
    the CPU oracle) use the torch composition of the reference modules below."""
    if head.is_cuda:
        from .adapter_hip import fused_gaussians_from_head
        return fused_gaussians_from_head(head, depths, images, extrinsics, intrinsics, adapter)
    return gaussians_from_head_torch(head, depths, images, extrinsics, intrinsics, adapter)


def gaussians_from_head_torch(head: torch.Tensor, depths: torch.Tensor, images: torch.Tensor,
                              extrinsics: torch.Tensor, intrinsics: torch.Tensor, adapter: GaussianAdapter):
    """gaussians_from_head as the reference's torch modules compute it (the fp32 reference of
    the fused kernel, and the host-tensor path)."""
    from .decoder import Gaussians

    B, V = extrinsics.shape[:2]
    h, w = images.shape[-2:]
    opac = head[..., :1].sigmoid().unsqueeze(-1)              # [B, V, HW, 1, 1]
    raw = head[..., 1:].unsqueeze(-2)                          # [B, V, HW, srf=1, C-1]
    xy_ray, _ = sample_image_grid((h, w), head.device)
    xy_ray = xy_ray.reshape(h * w, 1, 2)
    pixel = 1 / torch.tensor((w, h), dtype=torch.float32, device=head.device)
    xy_ray = xy_ray + (raw[..., :2].sigmoid() - 0.5) * pixel   # [B, V, HW, 1, 2]
    e = lambda t: t[:, :, None, None, None]  # noqa: E731  "b v i j -> b v () () () i j"
    out = adapter.forward_torch(e(extrinsics), e(intrinsics), xy_ray[..., None, :], depths, opac, raw[..., None, 2:],
                                (h, w), input_images=images)
    G = V * h * w
    return Gaussians(out.means.reshape(B, G, 3), out.covariances.reshape(B, G, 3, 3),
                     out.harmonics.reshape(B, G, 3, adapter.d_sh), out.opacities.reshape(B, G))
