"""Fused Gaussian adapter on the device.

Two entries, one kernel per direction each:
  * `adapter_forward_hip` — the reference operator `GaussianAdapter.forward(extrinsics,
    intrinsics, coordinates, depths, opacities, raw_gaussians, image_shape, eps, point_cloud,
    input_images)` (gaussian_adapter.py:49-102, called at encoder_depthsplat.py:300-314) on
    dga_adapter_forward / dga_adapter_backward; `GaussianAdapter.forward` routes device
    tensors here.
  * `fused_gaussians_from_head` — the encoder glue fused in front of it (opacity sigmoid,
    pixel offsets: encoder_depthsplat.py:224-346) on dga_adapter_fwd / dga_adapter_bwd,
    producing the decoder's Gaussians straight from the head channels.
Both replace ~30 torch kernels and batched 3x3 GEMMs per call (build_covariance,
get_world_rays, rotate_sh: gaussians.py:8-44, projection.py:91-114, sh_rotation.py:10-30).
Per-view constants (c2w rotation and translation, K^-1, Wigner-D blocks of the rotation) come
from dga_adapter_cameras, which solves the Wigner-D blocks exactly as sh_rotation.wigner_d.
"""
from __future__ import annotations

import torch

from . import _lib, raster
from .sh_rotation import _probe, wigner_d

CAM_FLOATS = 104  # R[9] t[3] Kinv[9] D1[9] D2[25] D3[49] (include/dsplat_hip.h)


_probe_cache: dict = {}


def _probes(device) -> torch.Tensor:
    """sh_rotation's probe directions and pseudo-inverses for l = 1..3 (float64, on device)."""
    key = str(device)
    t = _probe_cache.get(key)
    if t is None:
        parts = []
        for l in (1, 2, 3):
            pts, pinv = _probe(l)
            parts += [pts.reshape(-1), pinv.reshape(-1)]
        t = torch.cat(parts).to(torch.float64).to(device)
        _probe_cache[key] = t
    return t


def adapter_cameras(extrinsics: torch.Tensor, intrinsics: torch.Tensor, sh_degree: int) -> torch.Tensor:
    """[B, V, 4, 4] c2w + [B, V, 3, 3] normalised K -> [B*V, 104] float32 view blocks, built
    on the device in one kernel (dga_adapter_cameras)."""
    lib = _lib.load()
    B, V = extrinsics.shape[:2]
    ext = extrinsics.detach().reshape(B * V, 4, 4).contiguous().float()
    K = intrinsics.detach().reshape(B * V, 3, 3).contiguous().float()
    _lib.require_gpu(ext, K)
    cams = torch.empty((B * V, CAM_FLOATS), dtype=torch.float32, device=ext.device)
    _lib.check(lib.dga_adapter_cameras(B * V, ext.data_ptr(), K.data_ptr(), int(sh_degree),
                                       _probes(ext.device).data_ptr(), cams.data_ptr(), _lib.stream_of(ext.device)),
               "dga_adapter_cameras")
    return cams


def adapter_cameras_torch(extrinsics: torch.Tensor, intrinsics: torch.Tensor, sh_degree: int) -> torch.Tensor:
    """The same blocks from the torch functions the reference path uses (test reference)."""
    B, V = extrinsics.shape[:2]
    ext = extrinsics.detach().reshape(B * V, 4, 4).float()
    K = intrinsics.detach().reshape(B * V, 3, 3).float()
    R = ext[:, :3, :3]
    parts = [R.reshape(-1, 9), ext[:, :3, 3], K.inverse().reshape(-1, 9)]
    for l, n in ((1, 9), (2, 25), (3, 49)):
        if l <= sh_degree:
            parts.append(wigner_d(l, R).reshape(-1, n).float())
        else:
            parts.append(torch.zeros(B * V, n, device=ext.device))
    return torch.cat(parts, dim=1).contiguous()


class _FusedAdapter(torch.autograd.Function):
    @staticmethod
    def forward(ctx, head, depths, images, cams, smin, smax, sh_mask, d_sh):
        lib = _lib.load()
        _lib.require_gpu(head, depths, images, cams, sh_mask)
        B, V, HW, C = head.shape
        H, W = images.shape[-2:]
        G = V * HW
        dev = head.device
        means = torch.empty((B, G, 3), dtype=torch.float32, device=dev)
        cov = torch.empty((B, G, 3, 3), dtype=torch.float32, device=dev)
        harm = torch.empty((B, G, 3, d_sh), dtype=torch.float32, device=dev)
        opac = torch.empty((B, G), dtype=torch.float32, device=dev)
        _lib.check(raster._timed("k_adapter_fwd", lib.dga_adapter_fwd, B, V, H, W, d_sh, C, head.data_ptr(), depths.data_ptr(), images.data_ptr(),
                                       cams.data_ptr(), float(smin), float(smax), sh_mask.data_ptr(),
                                       means.data_ptr(), cov.data_ptr(), harm.data_ptr(), opac.data_ptr(),
                                       _lib.stream_of(dev)), "dga_adapter_fwd")
        ctx.save_for_backward(head, depths, cams, sh_mask)
        ctx.args = (smin, smax, d_sh, H, W)
        return means, cov, harm, opac

    @staticmethod
    def backward(ctx, dmeans, dcov, dharm, dopac):
        lib = _lib.load()
        head, depths, cams, sh_mask = ctx.saved_tensors
        smin, smax, d_sh, H, W = ctx.args
        B, V, HW, C = head.shape
        f = lambda t: None if t is None else t.contiguous().float()  # noqa: E731
        dmeans, dcov, dharm, dopac = f(dmeans), f(dcov), f(dharm), f(dopac)
        dhead = torch.empty_like(head)
        ddepth = torch.empty_like(depths) if ctx.needs_input_grad[1] else None
        p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        _lib.check(raster._timed("k_adapter_bwd", lib.dga_adapter_bwd, B, V, H, W, d_sh, C, head.data_ptr(), depths.data_ptr(), cams.data_ptr(),
                                       float(smin), float(smax), sh_mask.data_ptr(), p(dmeans), p(dcov), p(dharm),
                                       p(dopac), dhead.data_ptr(), p(ddepth), _lib.stream_of(head.device)),
                   "dga_adapter_bwd")
        return dhead, ddepth, None, None, None, None, None, None


def fused_gaussians_from_head(head, depths, images, extrinsics, intrinsics, adapter):
    """gaussians_from_head (gaussian_adapter.py) through the fused HIP kernels."""
    from .decoder import Gaussians

    B, V, HW, C = head.shape
    d_sh = adapter.d_sh
    if C < 10 + 3 * d_sh:
        raise ValueError(f"head has {C} channels; needs 3 + {adapter.d_in}")
    cams = adapter_cameras(extrinsics, intrinsics, adapter.cfg.sh_degree)
    depths_f = depths.reshape(B, V, HW)
    means, cov, harm, opac = _FusedAdapter.apply(
        head.contiguous().float(), depths_f.contiguous().float(), images.detach().contiguous().float(), cams,
        adapter.cfg.gaussian_scale_min, adapter.cfg.gaussian_scale_max,
        adapter.sh_mask.to(head.device).float().contiguous(), d_sh)
    return Gaussians(means, cov, harm, opac)


class _RefAdapter(torch.autograd.Function):
    """GaussianAdapter.forward on dga_adapter_forward / dga_adapter_backward. Gradients reach
    raw_gaussians, coordinates and depths; cameras and images get none (as in the fused
    encoder path; the reference's extrinsics / intrinsics / images are data)."""

    @staticmethod
    def forward(ctx, raw, coords, depths, images, cams, sh_mask, meta):
        lib = _lib.load()
        BV, H, W, S, d_sh, smin, smax, eps = meta
        N, C = raw.shape
        dev = raw.device
        means = torch.empty((N, 3), dtype=torch.float32, device=dev)
        cov = torch.empty((N, 3, 3), dtype=torch.float32, device=dev)
        harm = torch.empty((N, 3, d_sh), dtype=torch.float32, device=dev)
        scales = torch.empty((N, 3), dtype=torch.float32, device=dev)
        rots = torch.empty((N, 4), dtype=torch.float32, device=dev)
        _lib.check(lib.dga_adapter_forward(BV, H, W, S, d_sh, C, raw.data_ptr(), coords.data_ptr(), depths.data_ptr(),
                                           images.data_ptr(), cams.data_ptr(), float(smin), float(smax),
                                           sh_mask.data_ptr(), float(eps), means.data_ptr(), cov.data_ptr(),
                                           harm.data_ptr(), scales.data_ptr(), rots.data_ptr(), _lib.stream_of(dev)),
                   "dga_adapter_forward")
        ctx.save_for_backward(raw, coords, depths, cams, sh_mask)
        ctx.meta = meta
        return means, cov, harm, scales, rots

    @staticmethod
    def backward(ctx, dmeans, dcov, dharm, dscales, drots):
        lib = _lib.load()
        raw, coords, depths, cams, sh_mask = ctx.saved_tensors
        BV, H, W, S, d_sh, smin, smax, eps = ctx.meta
        N, C = raw.shape
        f = lambda t: None if t is None else t.contiguous().float()  # noqa: E731
        p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        g = [f(t) for t in (dmeans, dcov, dharm, dscales, drots)]
        draw = torch.empty_like(raw)
        dcoords = torch.empty_like(coords) if ctx.needs_input_grad[1] else None
        ddepth = torch.empty_like(depths) if ctx.needs_input_grad[2] else None
        _lib.check(lib.dga_adapter_backward(BV, H, W, S, d_sh, C, raw.data_ptr(), coords.data_ptr(), depths.data_ptr(),
                                            cams.data_ptr(), float(smin), float(smax), sh_mask.data_ptr(), float(eps),
                                            *[p(t) for t in g], draw.data_ptr(), p(dcoords), p(ddepth),
                                            _lib.stream_of(raw.device)), "dga_adapter_backward")
        return draw, dcoords, ddepth, None, None, None, None


def _per_view(t: torch.Tensor, b: int, v: int, tail: tuple, name: str) -> torch.Tensor:
    """[b, v, 1, ..., 1, *tail] (the reference's "b v i j -> b v () () () i j") -> [b*v, *tail].
    Leading dims of 1 broadcast as in the reference (one camera for every batch entry or
    view); a camera that varies per pixel is not representable by the fused kernel."""
    if t.dim() < len(tail) or tuple(t.shape[-len(tail):]) != tail:
        raise ValueError(f"{name} must end in {tail}; got {tuple(t.shape)}")
    lead = tuple(t.shape[:-len(tail)])
    lead = (1,) * max(0, 2 - len(lead)) + lead
    if lead[0] not in (1, b) or lead[1] not in (1, v) or any(d != 1 for d in lead[2:]):
        raise ValueError(f"{name} {tuple(t.shape)}: the fused adapter takes one camera per (batch, view), "
                         f"broadcastable to [{b}, {v}, 1, ..., 1, {', '.join(map(str, tail))}]")
    return t.reshape(lead[0], lead[1], *tail).expand(b, v, *tail).reshape(b * v, *tail)


def adapter_forward_hip(adapter, extrinsics, intrinsics, coordinates, depths, opacities, raw_gaussians, image_shape,
                        eps: float = 1e-8, input_images=None):
    """GaussianAdapter.forward (gaussian_adapter.py:49-102) for device tensors. Batch shape =
    opacities.shape = [b, v, h*w, *rest] (rest: surfaces x Gaussians per pixel)."""
    from .gaussian_adapter import AdapterGaussians

    if input_images is None:
        raise ValueError("GaussianAdapter.forward needs input_images (gaussian_adapter.py:69)")
    if intrinsics is None:
        raise ValueError("GaussianAdapter.forward needs intrinsics for the pixel rays")
    _lib.require_gpu(extrinsics, intrinsics, coordinates, depths, opacities, raw_gaussians, input_images)
    batch = tuple(opacities.shape)
    if len(batch) < 3:
        raise ValueError(f"opacities {batch}: expected [b, v, h*w, ...]")
    b, v, r = batch[:3]
    h, w = image_shape
    if r != h * w or tuple(input_images.shape) != (b, v, 3, h, w):
        raise ValueError(f"rays {r} / images {tuple(input_images.shape)} do not match image_shape {image_shape}")
    S = 1
    for d in batch[3:]:
        S *= d
    d_sh = adapter.d_sh
    C = raw_gaussians.shape[-1]
    if C < 7 + 3 * d_sh:
        raise ValueError(f"raw_gaussians has {C} channels; the adapter needs {adapter.d_in}")
    N = b * v * r * S
    f = lambda t: t.contiguous().float()  # noqa: E731
    raw = f(raw_gaussians.expand(*batch, C)).reshape(N, C)
    coords = f(coordinates.expand(*batch, 2)).reshape(N, 2)
    dep = f(depths.expand(*batch)).reshape(N)
    ext = _per_view(extrinsics, b, v, (4, 4), "extrinsics")
    K = _per_view(intrinsics, b, v, (3, 3), "intrinsics")
    cams = adapter_cameras(ext.view(b, v, 4, 4), K.view(b, v, 3, 3), adapter.cfg.sh_degree)
    meta = (b * v, h, w, S, d_sh, adapter.cfg.gaussian_scale_min, adapter.cfg.gaussian_scale_max, float(eps))
    means, cov, harm, scales, rots = _RefAdapter.apply(raw, coords, dep, f(input_images.detach()), cams,
                                                       adapter.sh_mask.to(raw.device).float().contiguous(), meta)
    return AdapterGaussians(means=means.view(*batch, 3), covariances=cov.view(*batch, 3, 3),
                            scales=scales.view(*batch, 3), rotations=rots.view(*batch, 4),
                            harmonics=harm.view(*batch, 3, d_sh), opacities=opacities)
