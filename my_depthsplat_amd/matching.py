"""Plane-sweep cost volume on MI355X: drop-in for the cost-volume block of
src/model/encoder/unimatch/ (SURVEY.md §8a rows A17-A20).

  coords_grid                        matching.py:5-21
  warp_with_pose_depth_candidates    matching.py:24-90 (same signature; HIP dcv_warp_fwd/bwd)
  batch_features_camera_parameters   mv_transformer.py:653-747
  depth_candidates                   mv_unimatch.py:416-475
  plane_sweep_cost_volume            NEW fused op = warp + correlation (mv_unimatch.py:484-505)
                                     without materialising [B, C, D, H, W] (HIP dcv_cost_volume_*)
"""
from __future__ import annotations

import torch
from einops import repeat

from . import _lib


def coords_grid(b, h, w, homogeneous=False, device=None):
    """[b, 2 or 3, h, w] integer pixel coordinates (x, y[, 1]) (matching.py:5-21)."""
    ys, xs = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    parts = [xs, ys] + ([torch.ones_like(xs)] if homogeneous else [])
    g = torch.stack(parts, dim=0).float()[None].repeat(b, 1, 1, 1)
    return g if device is None else g.to(device)


def _f(t):
    return t.contiguous().float()


class _Warp(torch.autograd.Function):
    @staticmethod
    def forward(ctx, feature, intrinsics, pose, depth, clamp):
        lib = _lib.load()
        B, C, H, W = feature.shape
        D = depth.shape[1]
        out = torch.empty((B, C, D, H, W), dtype=torch.float32, device=feature.device)
        _lib.check(lib.dcv_warp_fwd(B, C, H, W, D, feature.data_ptr(), intrinsics.data_ptr(), pose.data_ptr(),
                                    depth.data_ptr(), clamp, out.data_ptr(), _lib.stream_of(feature.device)),
                   "dcv_warp_fwd")
        ctx.save_for_backward(intrinsics, pose, depth)
        ctx.meta = (B, C, H, W, D, clamp)
        return out

    @staticmethod
    def backward(ctx, dout):
        intrinsics, pose, depth = ctx.saved_tensors
        B, C, H, W, D, clamp = ctx.meta
        dout = _f(dout)
        dfeat = torch.empty((B, C, H, W), dtype=torch.float32, device=dout.device)
        _lib.check(_lib.load().dcv_warp_bwd(B, C, H, W, D, dout.data_ptr(), intrinsics.data_ptr(), pose.data_ptr(),
                                            depth.data_ptr(), clamp, dfeat.data_ptr(), _lib.stream_of(dout.device)),
                   "dcv_warp_bwd")
        return dfeat, None, None, None, None


def warp_with_pose_depth_candidates(feature1, intrinsics, pose, depth, clamp_min_depth=1e-3,
                                    grid_sample_disable_cudnn=False):
    """feature1 [B,C,H,W], intrinsics [B,3,3], pose [B,4,4], depth [B,D,H,W] -> [B,C,D,H,W]
    (matching.py:24-90). Geometry gets no gradient; feature1 does."""
    if not (intrinsics.size(1) == intrinsics.size(2) == 3):
        raise ValueError("intrinsics must be [B, 3, 3]")
    if not (pose.size(1) == pose.size(2) == 4):
        raise ValueError("pose must be [B, 4, 4]")
    if depth.dim() != 4:
        raise ValueError("depth must be [B, D, H, W]")
    _lib.require_gpu(feature1, intrinsics, pose, depth)
    return _Warp.apply(_f(feature1), _f(intrinsics).detach(), _f(pose).detach(), _f(depth).detach(),
                       float(clamp_min_depth))


def _cost_volume_fwd(ref, tgt, intrinsics, pose, depth, per_pixel, clamp):
    lib = _lib.load()
    B, J, C, H, W = tgt.shape
    D = depth.shape[1]
    dev = ref.device
    # the kernel path, chosen once: the backward is handed the same one (include/dsplat_hip.h)
    path = lib.dcv_cost_volume_path(B, J, C, H, W)
    # channel-last copies of the features + the epipolar pixel groups (the backward reuses
    # them; after a band-kernel forward the backward makes them)
    ws = torch.empty(lib.dcv_cost_volume_workspace_size(B, J, C, H, W), dtype=torch.uint8, device=dev)
    cost = torch.empty((B, D, H, W), dtype=torch.float32, device=dev)
    _lib.check(lib.dcv_cost_volume_fwd(B, J, C, H, W, D, int(per_pixel), path, ref.data_ptr(), tgt.data_ptr(),
                                       intrinsics.data_ptr(), pose.data_ptr(), depth.data_ptr(), clamp,
                                       ws.data_ptr(), cost.data_ptr(), _lib.stream_of(dev)), "dcv_cost_volume_fwd")
    return cost, ws, path


class _CostVolume(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ref, tgt, intrinsics, pose, depth, per_pixel, clamp):
        B, J, C, H, W = tgt.shape
        D = depth.shape[1]
        cost, ws, path = _cost_volume_fwd(ref, tgt, intrinsics, pose, depth, per_pixel, clamp)
        ctx.save_for_backward(ref, tgt, ws, intrinsics, pose, depth)
        ctx.meta = (B, J, C, H, W, D, per_pixel, clamp, path)
        return cost

    @staticmethod
    def backward(ctx, dcost):
        ref, tgt, ws, intrinsics, pose, depth = ctx.saved_tensors
        B, J, C, H, W, D, per_pixel, clamp, path = ctx.meta
        dev = ref.device
        dcost = _f(dcost)
        dref = torch.empty_like(ref)
        dtgt = torch.empty((B, J, C, H, W), dtype=torch.float32, device=dev)
        lib = _lib.load()
        scratch = torch.empty(lib.dcv_cost_volume_bwd_workspace_size(B, J, C, H, W), dtype=torch.uint8, device=dev)
        _lib.check(lib.dcv_cost_volume_bwd(
            B, J, C, H, W, D, int(per_pixel), path, ref.data_ptr(), tgt.data_ptr(), ws.data_ptr(), intrinsics.data_ptr(),
            pose.data_ptr(), depth.data_ptr(), clamp, dcost.data_ptr(), dref.data_ptr(), dtgt.data_ptr(),
            scratch.data_ptr(), _lib.stream_of(dev)), "dcv_cost_volume_bwd")
        return dref, dtgt, None, None, None, None, None


def plane_sweep_cost_volume(ref: torch.Tensor, tgt: torch.Tensor, intrinsics: torch.Tensor, pose: torch.Tensor,
                            depth: torch.Tensor, clamp_min_depth: float = 1e-3) -> torch.Tensor:
    """Fused warp + correlation (mv_unimatch.py:484-505):
    cost[b,d,y,x] = mean_j( sum_c ref[b,c,y,x] * warp(tgt[b,j])[c,d,y,x] ) / sqrt(C).
    ref [B,C,H,W]; tgt [B,J,C,H,W]; intrinsics [B,3,3] or [B,J,3,3] (pixel units at this
    scale, the reference uses the ref-view K for every source view); pose [B,J,4,4]
    (= tgt_c2w^-1 ref_c2w); depth [B,D] (per-image candidates, scale 0) or [B,D,H,W]
    (per-pixel candidates, scale > 0) -- DEPTH values, not inverse depth. -> [B,D,H,W]."""
    B, J, C, H, W = tgt.shape
    if ref.shape != (B, C, H, W):
        raise ValueError(f"ref {tuple(ref.shape)} does not match tgt {tuple(tgt.shape)}")
    if intrinsics.dim() == 3:
        intrinsics = intrinsics[:, None].expand(B, J, 3, 3)
    if depth.dim() not in (2, 4):
        raise ValueError("depth must be [B, D] or [B, D, H, W]")
    _lib.require_gpu(ref, tgt, intrinsics, pose, depth)
    per_pixel = depth.dim() == 4
    args = (_f(ref), _f(tgt), _f(intrinsics).detach(), _f(pose).detach(), _f(depth).detach(), per_pixel,
            float(clamp_min_depth))
    if torch.is_grad_enabled() and (args[0].requires_grad or args[1].requires_grad):
        return _CostVolume.apply(*args)
    # nothing to differentiate: the launch without the autograd node (its set-up is ~5 us of host
    # time, a third of a 32x32 call)
    return _cost_volume_fwd(*args)[0]


class _CostVolumeViews(torch.autograd.Function):
    """dcv_cost_volume_views_fwd / _bwd (include/dsplat_hip.h): features read once."""

    @staticmethod
    def forward(ctx, features, nn, intrinsics, pose, depth, per_pixel, clamp, fanin):
        lib = _lib.load()
        BV, C, H, W = features.shape
        J, D = nn.shape[1], depth.shape[1]
        dev = features.device
        ws = torch.empty(lib.dcv_cost_volume_views_workspace_size(BV, J, C, H, W), dtype=torch.uint8, device=dev)
        cost = torch.empty((BV, D, H, W), dtype=torch.float32, device=dev)
        _lib.check(lib.dcv_cost_volume_views_fwd(BV, J, C, H, W, D, int(per_pixel), features.data_ptr(), nn.data_ptr(),
                                                 intrinsics.data_ptr(), pose.data_ptr(), depth.data_ptr(), clamp,
                                                 ws.data_ptr(), cost.data_ptr(), _lib.stream_of(dev)),
                   "dcv_cost_volume_views_fwd")
        ctx.save_for_backward(features, nn, ws, intrinsics, pose, depth)
        ctx.meta = (BV, J, C, H, W, D, per_pixel, clamp, fanin)
        return cost

    @staticmethod
    def backward(ctx, dcost):
        features, nn, ws, intrinsics, pose, depth = ctx.saved_tensors
        BV, J, C, H, W, D, per_pixel, clamp, fanin = ctx.meta
        dev = features.device
        dcost = _f(dcost)
        lib = _lib.load()
        dfeat = torch.empty_like(features)
        scratch = torch.empty(lib.dcv_cost_volume_views_bwd_workspace_size(BV, J, C, H, W), dtype=torch.uint8,
                              device=dev)
        _lib.check(lib.dcv_cost_volume_views_bwd(
            BV, J, C, H, W, D, int(per_pixel), fanin, features.data_ptr(), nn.data_ptr(), ws.data_ptr(),
            intrinsics.data_ptr(), pose.data_ptr(), depth.data_ptr(), clamp, dcost.data_ptr(), dfeat.data_ptr(),
            scratch.data_ptr(), _lib.stream_of(dev)), "dcv_cost_volume_views_bwd")
        return dfeat, None, None, None, None, None, None, None


def plane_sweep_cost_volume_views(features: torch.Tensor, nn: torch.Tensor, intrinsics: torch.Tensor,
                                  pose: torch.Tensor, depth: torch.Tensor, clamp_min_depth: float = 1e-3,
                                  max_fanin: int | None = None) -> torch.Tensor:
    """plane_sweep_cost_volume(features, features[nn], ...) without the stacked copy:
    features [BV,C,H,W] (every view's features, once), nn [BV,J] integer indices into BV (view
    b's J source views: the reference's nn_matrix gather, mv_transformer.py:653-747, flattened
    over the batch), intrinsics [BV,3,3] or [BV,J,3,3], pose [BV,J,4,4], depth [BV,D] or
    [BV,D,H,W] -> cost [BV,D,H,W]; the gradient reaches `features` through both roles.
    Matrix-core sizes (dcv_cost_volume_path == epipolar groups) run the views kernels; other
    sizes gather tgt and take plane_sweep_cost_volume (both HIP). max_fanin: an upper bound on
    how often one view appears in nn (taken from nn when it is a CPU tensor)."""
    BV, C, H, W = features.shape
    if nn.dim() != 2 or nn.shape[0] != BV:
        raise ValueError(f"nn must be [BV={BV}, J], got {tuple(nn.shape)}")
    J = nn.shape[1]
    if not nn.is_cuda:
        if nn.numel() and (int(nn.min()) < 0 or int(nn.max()) >= BV):
            raise ValueError(f"nn indices must lie in [0, {BV})")
        if max_fanin is None and nn.numel():
            max_fanin = int(torch.bincount(nn.flatten().long(), minlength=BV).max())
    lib = _lib.load()
    if lib.dcv_cost_volume_path(BV, J, C, H, W) != 1:  # band / direct sizes: the stacked path
        nn_d = nn.to(features.device).long()
        return plane_sweep_cost_volume(features, features[nn_d], intrinsics, pose, depth, clamp_min_depth)
    if intrinsics.dim() == 3:
        intrinsics = intrinsics[:, None].expand(BV, J, 3, 3)
    if depth.dim() not in (2, 4):
        raise ValueError("depth must be [B, D] or [B, D, H, W]")
    _lib.require_gpu(features, intrinsics, pose, depth)
    nn32 = nn.to(device=features.device, dtype=torch.int32).contiguous()
    return _CostVolumeViews.apply(_f(features), nn32, _f(intrinsics).detach(), _f(pose).detach(), _f(depth).detach(),
                                  depth.dim() == 4, float(clamp_min_depth), int(max_fanin or 0))


def batch_features_camera_parameters(features, intrinsics, extrinsics, nn_matrix=None, no_batch=False):
    """Reference view + its source views for every view (mv_transformer.py:653-747).
    features/intrinsics/extrinsics: lists over views of [B,C,H,W] / [B,3,3] / [B,4,4].
    Returns ref [BV,C,H,W], ref K, ref c2w, tgt [BV,V-1,C,H,W], tgt K, tgt c2w.

    Token features [B,HW,C] per view (the reference's `features_tensor.dim() == 4` branch,
    mv_transformer.py:706-708: the nn_matrix gather over "b v -> b v hw c") are accepted too.
    The reference reaches that branch only with its entry assert disabled and then only
    returns lists (no_batch; its batched return unpacks C, H, W); here the batched return
    stacks them as ref [BV,HW,C] and tgt [BV,n,HW,C]."""
    V = len(features)
    if features[0].dim() not in (3, 4) or intrinsics[0].dim() != 3 or extrinsics[0].dim() != 3:
        raise ValueError("features must be [B,C,H,W] (or [B,HW,C] tokens), intrinsics [B,3,3], extrinsics [B,4,4]")
    if nn_matrix is not None:
        F_ = torch.stack(features, 1)
        K_ = torch.stack(intrinsics, 1)
        E_ = torch.stack(extrinsics, 1)
        n_sel = nn_matrix.size(-1) - 1
    else:
        n_sel = V - 1
    q, qk, qe, kv, kvk, kve = [], [], [], [], [], []
    for i in range(V):
        q.append(features[i])
        qk.append(intrinsics[i])
        qe.append(extrinsics[i])
        if nn_matrix is not None:
            sel = nn_matrix[:, i, 1:]
            if F_.dim() == 5:
                c, h, w = F_.shape[-3:]
                idx = repeat(sel, "b v -> b v c h w", c=c, h=h, w=w)
            else:
                hw, c = F_.shape[-2:]
                idx = repeat(sel, "b v -> b v hw c", hw=hw, c=c)
            kv.append(torch.gather(F_, 1, idx))
            kvk.append(torch.gather(K_, 1, repeat(sel, "b v -> b v i j", i=3, j=3)))
            kve.append(torch.gather(E_, 1, repeat(sel, "b v -> b v i j", i=4, j=4)))
        else:
            others = [j for j in range(V) if j != i]
            kv.append(torch.stack([features[j] for j in others], 1))
            kvk.append(torch.stack([intrinsics[j] for j in others], 1))
            kve.append(torch.stack([extrinsics[j] for j in others], 1))
    if no_batch:
        return q, qk, qe, kv, kvk, kve
    fs = tuple(q[0].shape[1:])
    return (torch.stack(q, 1).reshape(-1, *fs), torch.stack(qk, 1).reshape(-1, 3, 3),
            torch.stack(qe, 1).reshape(-1, 4, 4), torch.stack(kv, 1).reshape(-1, n_sel, *fs),
            torch.stack(kvk, 1).reshape(-1, n_sel, 3, 3), torch.stack(kve, 1).reshape(-1, n_sel, 4, 4))


def depth_candidates(min_depth: torch.Tensor, max_depth: torch.Tensor, num_candidates: int, scale_idx: int = 0,
                     depth: torch.Tensor | None = None) -> torch.Tensor:
    """Inverse-depth hypotheses (mv_unimatch.py:416-461). min/max_depth are INVERSE depths [BV].
    scale 0: [BV, D, 1, 1] linspace per image; scale s > 0: [BV, D/4^s, H, W] per-pixel window
    around the (inverse) `depth` [BV, 1, H, W] of the previous scale, clamped to [min, max]."""
    D = num_candidates // (4 ** scale_idx)
    lin = torch.linspace(0, 1, D, dtype=min_depth.dtype, device=min_depth.device).view(1, D, 1, 1)
    if scale_idx == 0:
        return min_depth.view(-1, 1, 1, 1) + lin * (max_depth - min_depth).view(-1, 1, 1, 1)
    interval = ((max_depth - min_depth) / (num_candidates - 1) / (2 ** scale_idx)).view(-1, 1, 1, 1)
    lo = (depth - interval * (D // 2)).clamp(min=min_depth.view(-1, 1, 1, 1))
    hi = (depth + interval * (D // 2 - 1)).clamp(max=max_depth.view(-1, 1, 1, 1))
    return lo + lin * (hi - lo)
