"""Fused Gaussian adapter on the device (dga_adapter_fwd / dga_adapter_bwd).

Replaces the encoder glue + GaussianAdapter + rotate_sh chain (encoder_depthsplat.py:224-346,
gaussian_adapter.py:49-102, gaussians.py:8-44, sh_rotation.py:10-30) — ~30 torch kernels and
batched 3x3 GEMMs per call — by one kernel per direction. Per-view constants (c2w rotation
and translation, K^-1, Wigner-D blocks of the rotation) are built here with the same torch
functions the reference path uses, so both paths rotate SH with identical matrices.
"""
from __future__ import annotations

import torch

from . import _lib
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
        _lib.check(lib.dga_adapter_fwd(B, V, H, W, d_sh, C, head.data_ptr(), depths.data_ptr(), images.data_ptr(),
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
        _lib.check(lib.dga_adapter_bwd(B, V, H, W, d_sh, C, head.data_ptr(), depths.data_ptr(), cams.data_ptr(),
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
