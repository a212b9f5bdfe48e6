"""Drop-in for src/model/decoder/cuda_splatting.py on MI355X.

Same function names, signatures, argument meaning and return shapes as the reference:
  get_projection_matrix     cuda_splatting.py:16-43
  render_cuda               cuda_splatting.py:46-126
  render_cuda_orthographic  cuda_splatting.py:129-219
  render_depth_cuda         cuda_splatting.py:225-264
plus `render_views`, the batched entry the decoder uses (one scene's Gaussians shared by
many target views, no per-view repeat, no per-view Python loop).

The camera set-up below (scale-invariant rescale, fov -> tan, projection / view matrix
transposes, campos, triu covariance gather, SH layout) restates the reference wrapper
line by line; it is pinned by tests/golden/cuda_splatting_settings.npz, which records the
exact tensors the reference hands to its rasterizer. The rasterization itself runs in
libdsplat_hip.so (my_depthsplat_amd/raster.py).
"""
from __future__ import annotations

import math
from typing import Literal

import torch

from . import raster
from .projection import get_fov, homogenize_points

DepthRenderingMode = Literal["depth", "disparity", "relative_disparity", "log"]

_TRIU_ROW = (0, 0, 0, 1, 1, 2)
_TRIU_COL = (0, 1, 2, 1, 2, 2)


def get_projection_matrix(near: torch.Tensor, far: torch.Tensor, fov_x: torch.Tensor,
                          fov_y: torch.Tensor) -> torch.Tensor:
    """Frustum -> x, y in (-1, 1), z in (0, 1) (cuda_splatting.py:16-43)."""
    tx = (0.5 * fov_x).tan()
    ty = (0.5 * fov_y).tan()
    top = ty * near
    bottom = -top
    right = tx * near
    left = -right
    (b,) = near.shape
    m = torch.zeros((b, 4, 4), dtype=torch.float32, device=near.device)
    m[:, 0, 0] = 2 * near / (right - left)
    m[:, 1, 1] = 2 * near / (top - bottom)
    m[:, 0, 2] = (right + left) / (right - left)
    m[:, 1, 2] = (top + bottom) / (top - bottom)
    m[:, 3, 2] = 1
    m[:, 2, 2] = far / (far - near)
    m[:, 2, 3] = -(far * near) / (far - near)
    return m


def camera_settings(extrinsics: torch.Tensor, intrinsics: torch.Tensor, near: torch.Tensor,
                    far: torch.Tensor, scale_invariant: bool = True) -> dict[str, torch.Tensor]:
    """Per-view rasterizer settings exactly as render_cuda builds them
    (cuda_splatting.py:62-86, 98-111). Returns viewmatrix / projmatrix ([b,4,4], already
    transposed), campos [b,3], tanfovx/tanfovy [b], and `scale` [b] (1/near or 1) that the
    kernels apply to the Gaussians (means * scale, covariances * scale^2)."""
    b = extrinsics.shape[0]
    if scale_invariant:
        scale = 1 / near
        extrinsics = extrinsics.clone()
        extrinsics[..., :3, 3] = extrinsics[..., :3, 3] * scale[:, None]
        near = near * scale
        far = far * scale
    else:
        scale = torch.ones(b, dtype=torch.float32, device=extrinsics.device)
    fov_x, fov_y = get_fov(intrinsics).unbind(dim=-1)
    tan_x = (0.5 * fov_x).tan()
    tan_y = (0.5 * fov_y).tan()
    proj = get_projection_matrix(near, far, fov_x, fov_y).transpose(1, 2)
    view = extrinsics.inverse().transpose(1, 2)
    full = view @ proj
    return {"viewmatrix": view, "projmatrix": full, "campos": extrinsics[:, :3, 3], "tanfovx": tan_x,
            "tanfovy": tan_y, "scale": scale}


def _cov6(cov: torch.Tensor) -> torch.Tensor:
    # cov[..., row, col] with (row, col) = torch.triu_indices(3, 3): xx xy xz yy yz zz
    # (cuda_splatting.py:114,122); backward puts gradient on the upper triangle only.
    return cov[..., list(_TRIU_ROW), list(_TRIU_COL)]


def render_views(extrinsics: torch.Tensor, intrinsics: torch.Tensor, near: torch.Tensor, far: torch.Tensor,
                 image_shape: tuple[int, int], background_color: torch.Tensor, gaussian_means: torch.Tensor,
                 gaussian_covariances: torch.Tensor, gaussian_sh_coefficients: torch.Tensor,
                 gaussian_opacities: torch.Tensor, view_scene: list[int], scale_invariant: bool = True,
                 use_sh: bool = True, return_radii: bool = False, ctx: "raster.RasterContext | None" = None):
    """Render V views of S scenes in one batch. extrinsics/intrinsics [V,4,4]/[V,3,3],
    near/far [V], background [V,3]; Gaussians per SCENE: means [S,G,3], covariances
    [S,G,3,3], harmonics [S,G,3,d_sh], opacities [S,G]; view_scene[v] in [0, S).
    Equivalent to render_cuda on the per-view repeated Gaussians. -> [V,3,H,W].
    ctx: the caller's raster.RasterContext (a decoder passes its own)."""
    if not (use_sh or gaussian_sh_coefficients.shape[-1] == 1):
        raise ValueError("use_sh=False needs harmonics with d_sh == 1 (cuda_splatting.py:60)")
    V = extrinsics.shape[0]
    h, w = image_shape
    n = gaussian_sh_coefficients.shape[-1]
    degree = math.isqrt(n) - 1
    try:
        return _render_views(extrinsics, intrinsics, near, far, image_shape, background_color, gaussian_means,
                             gaussian_covariances, gaussian_sh_coefficients, gaussian_opacities, view_scene,
                             scale_invariant, use_sh, return_radii, degree, ctx)
    except raster.EntryOverflow:
        if V == 1:
            raise
    # more (view, tile, Gaussian) entries than 32-bit offsets address: render the views in halves
    k = V // 2
    parts = [render_views(extrinsics[sl], intrinsics[sl], near[sl], far[sl], image_shape, background_color[sl]
                          if background_color.dim() > 1 else background_color, gaussian_means, gaussian_covariances,
                          gaussian_sh_coefficients, gaussian_opacities, list(view_scene[sl]),
                          scale_invariant=scale_invariant, use_sh=use_sh, return_radii=return_radii, ctx=ctx)
             for sl in (slice(0, k), slice(k, V))]
    if return_radii:
        return torch.cat([p[0] for p in parts]), torch.cat([p[1] for p in parts])
    return torch.cat(parts)


def _render_views(extrinsics, intrinsics, near, far, image_shape, background_color, gaussian_means,
                  gaussian_covariances, gaussian_sh_coefficients, gaussian_opacities, view_scene, scale_invariant,
                  use_sh, return_radii, degree, ctx=None):
    V = extrinsics.shape[0]
    h, w = image_shape
    # the camera_settings() math runs on the device (no torch op chain, no host sync): in one
    # launch that also zeroes the binning counters, or, for eager inference, inside the
    # binning kernel itself
    cams = raster.camera_inputs(extrinsics, intrinsics, near, far, background_color.expand(V, 3), view_scene,
                                scale_invariant)
    # The kernels read the decoder's layouts directly: harmonics [S,G,3,d_sh] (no
    # "b g xyz n -> b g n xyz" copy) and full covariances through the triu gather (no
    # [S,G,6] copy); gradients come back in the same layouts (upper triangle for cov).
    feats = gaussian_sh_coefficients if use_sh else gaussian_sh_coefficients[..., 0]
    color, radii = raster.rasterize_views(
        gaussian_means, feats, gaussian_opacities, gaussian_covariances, cams, view_scene,
        use_sh=use_sh, sh_degree=degree, image_height=h, image_width=w, channel_major_sh=True, ctx=ctx)
    return (color, radii) if return_radii else color


def render_cuda(extrinsics: torch.Tensor, intrinsics: torch.Tensor, near: torch.Tensor, far: torch.Tensor,
                image_shape: tuple[int, int], background_color: torch.Tensor, gaussian_means: torch.Tensor,
                gaussian_covariances: torch.Tensor, gaussian_sh_coefficients: torch.Tensor,
                gaussian_opacities: torch.Tensor, scale_invariant: bool = True,
                use_sh: bool = True, ctx: "raster.RasterContext | None" = None) -> torch.Tensor:
    """cuda_splatting.py:46-126: view i renders Gaussian set i. -> [b,3,H,W].
    (ctx, optional and last: the caller's raster.RasterContext.)"""
    b = extrinsics.shape[0]
    return render_views(extrinsics, intrinsics, near, far, image_shape, background_color, gaussian_means,
                        gaussian_covariances, gaussian_sh_coefficients, gaussian_opacities, list(range(b)),
                        scale_invariant=scale_invariant, use_sh=use_sh, ctx=ctx)


def orthographic_settings(extrinsics: torch.Tensor, width: torch.Tensor, height: torch.Tensor, near: torch.Tensor,
                          far: torch.Tensor, fov_degrees: float = 0.1, dump: dict | None = None) -> dict:
    """Pseudo-orthographic camera: tiny fov, camera pulled back by 0.5 width / tan(fov/2)
    (cuda_splatting.py:146-175). Returns the rasterizer settings per view."""
    b = extrinsics.shape[0]
    dev = extrinsics.device
    fov_x = torch.tensor(fov_degrees, device=dev).deg2rad()
    tan_x = (0.5 * fov_x).tan()
    dist = (0.5 * width) / tan_x
    tan_y = 0.5 * height / dist
    fov_y = (2 * tan_y).atan()
    near = near + dist
    far = far + dist
    move_back = torch.eye(4, dtype=torch.float32, device=dev)
    move_back[2, 3] = -dist  # as in the reference: one shared pull-back (b = 1 in practice)
    extrinsics = extrinsics @ move_back
    if dump is not None:
        dump.update(extrinsics=extrinsics, fov_x=fov_x, fov_y=fov_y, near=near, far=far)
    proj = get_projection_matrix(near, far, fov_x.expand(b), fov_y).transpose(1, 2)
    view = extrinsics.inverse().transpose(1, 2)
    return {"viewmatrix": view, "projmatrix": view @ proj, "campos": extrinsics[:, :3, 3],
            "tanfovx": tan_x.expand(b), "tanfovy": tan_y.expand(b) if tan_y.dim() == 0 else tan_y,
            "scale": torch.ones(b, dtype=torch.float32, device=dev)}


def render_cuda_orthographic(extrinsics: torch.Tensor, width: torch.Tensor, height: torch.Tensor,
                             near: torch.Tensor, far: torch.Tensor, image_shape: tuple[int, int],
                             background_color: torch.Tensor, gaussian_means: torch.Tensor,
                             gaussian_covariances: torch.Tensor, gaussian_sh_coefficients: torch.Tensor,
                             gaussian_opacities: torch.Tensor, fov_degrees: float = 0.1, use_sh: bool = True,
                             dump: dict | None = None) -> torch.Tensor:
    """cuda_splatting.py:129-219. -> [b,3,H,W]."""
    b = extrinsics.shape[0]
    h, w = image_shape
    if not (use_sh or gaussian_sh_coefficients.shape[-1] == 1):
        raise ValueError("use_sh=False needs harmonics with d_sh == 1")
    degree = math.isqrt(gaussian_sh_coefficients.shape[-1]) - 1
    st = orthographic_settings(extrinsics, width, height, near, far, fov_degrees, dump)
    scene = torch.arange(b, dtype=torch.int32, device=extrinsics.device)
    cams = raster.pack_cameras(st["viewmatrix"], st["projmatrix"], st["campos"], st["tanfovx"], st["tanfovy"],
                               background_color, scene)
    shs = gaussian_sh_coefficients.transpose(-1, -2)
    feats = shs if use_sh else shs[:, :, 0, :]
    color, _ = raster.rasterize_views(gaussian_means, feats, gaussian_opacities, _cov6(gaussian_covariances), cams,
                                      list(range(b)), use_sh=use_sh, sh_degree=degree, image_height=h,
                                      image_width=w)
    return color


def depth_colors(extrinsics: torch.Tensor, gaussian_means: torch.Tensor, near: torch.Tensor, far: torch.Tensor,
                 mode: DepthRenderingMode = "depth") -> torch.Tensor:
    """Per-view Gaussian colour used by render_depth_cuda (cuda_splatting.py:237-246): camera-
    space z, 1/z, or log(z.minimum(near).maximum(far)) (order as written). -> [b, g]."""
    cam_pts = torch.einsum("bij,bgj->bgi", extrinsics.inverse(), homogenize_points(gaussian_means))
    fake = cam_pts[..., 2]
    if mode == "disparity":
        fake = 1 / fake
    elif mode == "log":
        fake = fake.minimum(near[:, None]).maximum(far[:, None]).log()
    return fake


def render_depth_cuda(extrinsics: torch.Tensor, intrinsics: torch.Tensor, near: torch.Tensor, far: torch.Tensor,
                      image_shape: tuple[int, int], gaussian_means: torch.Tensor,
                      gaussian_covariances: torch.Tensor, gaussian_opacities: torch.Tensor,
                      scale_invariant: bool = True, mode: DepthRenderingMode = "depth",
                      ctx: "raster.RasterContext | None" = None) -> torch.Tensor:
    """Depth / disparity / log-depth as colour (cuda_splatting.py:225-264). -> [b,H,W]."""
    fake = depth_colors(extrinsics, gaussian_means, near, far, mode)
    b = fake.shape[0]
    out = render_cuda(extrinsics, intrinsics, near, far, image_shape,
                      torch.zeros((b, 3), dtype=fake.dtype, device=fake.device), gaussian_means,
                      gaussian_covariances, fake[..., None, None].expand(-1, -1, 3, 1), gaussian_opacities,
                      scale_invariant=scale_invariant, use_sh=False, ctx=ctx)
    return out.mean(dim=1)
