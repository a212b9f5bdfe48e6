"""Training-step fusion of the adapter and the rasterizer (round 6): head channels -> rendered
target views in one autograd node, so the backward runs the rasterizer's K7 and then ONE kernel
for K8 + K9 and the adapter's backward (dsr_head_bwd, include/dsplat_hip.h).

The reference trains through encoder glue -> GaussianAdapter -> decoder (encoder_depthsplat.py:
224-346, gaussian_adapter.py:49-102, decoder_splatting_cuda.py:35-67); its Gaussians are an
intermediate with exactly one consumer, the decoder. As separate drop-in modules
(gaussians_from_head + DecoderSplattingCUDA) the Gaussian gradients are written by the
rasterizer's preprocess backward and read back by the adapter's backward (~320 B per Gaussian);
here they stay in registers. The values are the two-module path's bit for bit
(tests/test_head_render.py): the same kernels up to K7, the same float operations after it.

`render_from_head` needs the fused adapter's inputs (device tensors, H*W a multiple of 256);
otherwise it composes gaussians_from_head and the decoder (same results, two backward kernels).
"""
from __future__ import annotations

import torch

from . import _lib, raster
from .adapter_hip import adapter_cameras


class _HeadRender(torch.autograd.Function):
    @staticmethod
    def forward(ctx, head, depths, images, acams, smin, smax, sh_mask, d_sh, tcams, view_scene, Ht, Wt, rctx):
        lib = _lib.load()
        B, V, HW, C = head.shape
        h, w = images.shape[-2:]
        G = V * HW
        dev = head.device
        means = torch.empty((B, G, 3), dtype=torch.float32, device=dev)
        cov = torch.empty((B, G, 3, 3), dtype=torch.float32, device=dev)
        harm = torch.empty((B, G, 3, d_sh), dtype=torch.float32, device=dev)
        opac = torch.empty((B, G), dtype=torch.float32, device=dev)
        _lib.check(raster._timed("k_adapter_fwd", lib.dga_adapter_fwd, B, V, h, w, d_sh, C, head.data_ptr(),
                                 depths.data_ptr(), images.data_ptr(), acams.data_ptr(), float(smin), float(smax),
                                 sh_mask.data_ptr(), means.data_ptr(), cov.data_ptr(), harm.data_ptr(), opac.data_ptr(),
                                 _lib.stream_of(dev)), "dga_adapter_fwd")
        Vt = len(view_scene)
        layout = raster.input_layout(harm, cov, True, True)
        dgeom = torch.empty((Vt, G, raster.DGEOM_WORDS), dtype=torch.int64, device=dev)
        color, state = raster.forward_raw(means, harm, True, raster.sh_degree_of(d_sh), opac, cov, tcams, Vt, Ht, Wt,
                                          layout, None, need_state=True, dgeom_zero=dgeom, ctx=rctx)
        state.dgeom = dgeom
        ctx.save_for_backward(head, depths, images, acams, sh_mask)
        ctx.state = state
        ctx.meta = (smin, smax, d_sh, h, w, G, list(view_scene), Ht, Wt)
        return color

    @staticmethod
    def backward(ctx, dcolor):
        lib = _lib.load()
        head, depths, images, acams, sh_mask = ctx.saved_tensors
        smin, smax, d_sh, h, w, G, view_scene, Ht, Wt = ctx.meta
        state, ctx.state = ctx.state, None
        B, V, HW, C = head.shape
        dev = head.device
        dgeom_fx, gscale = raster.render_bwd_raw(state, state.cams, dcolor, G)
        idx = raster.scene_view_index(view_scene, B, dev)
        dhead = torch.empty_like(head)
        ddepth = torch.empty_like(depths) if ctx.needs_input_grad[1] else None
        _lib.check(raster._timed("k_head_bwd", lib.dsr_head_bwd, B, V, h, w, d_sh, C, head.data_ptr(),
                                 depths.data_ptr(), images.data_ptr(), acams.data_ptr(), float(smin), float(smax),
                                 sh_mask.data_ptr(), Ht,
                                 Wt, state.cams.data_ptr(), state.geom.data_ptr(), dgeom_fx.data_ptr(),
                                 gscale.data_ptr(), idx.data_ptr(), idx[B + 1:].data_ptr(),
                                 raster._ptr(state.row_live), dhead.data_ptr(), raster._ptr(ddepth),
                                 _lib.stream_of(dev)), "dsr_head_bwd")
        return dhead, ddepth, None, None, None, None, None, None, None, None, None, None, None


def fusable(head: torch.Tensor, images: torch.Tensor, adapter) -> bool:
    """The fused node applies: device tensors, one Gaussian per pixel rows of >= 10 + 3 d_sh
    channels, and H*W a multiple of 256 (a workgroup's rows share one view)."""
    B, V, HW, C = head.shape
    return (head.is_cuda and images.is_cuda and HW % 256 == 0 and adapter.d_sh in (1, 4, 9, 16)
            and C >= 10 + 3 * adapter.d_sh)


def render_from_head(decoder, head: torch.Tensor, depths: torch.Tensor, images: torch.Tensor,
                     extrinsics: torch.Tensor, intrinsics: torch.Tensor, adapter, tgt_extrinsics: torch.Tensor,
                     tgt_intrinsics: torch.Tensor, near: torch.Tensor, far: torch.Tensor,
                     image_shape: tuple[int, int]) -> torch.Tensor:
    """decoder(gaussians_from_head(head, depths, images, extrinsics, intrinsics, adapter),
    tgt_extrinsics, tgt_intrinsics, near, far, image_shape).color as one autograd node.
    head [B, V, H*W, C]; depths [B, V, H*W, 1, 1]; images [B, V, 3, H, W]; extrinsics /
    intrinsics [B, V, 4, 4] / [B, V, 3, 3] (context views, c2w, normalised K); tgt_* [B, v, ...];
    near / far [B, v] -> colour [B, v, 3, h, w]. Gradients for head (and depths)."""
    from .gaussian_adapter import gaussians_from_head
    if not fusable(head, images, adapter):
        g = gaussians_from_head(head, depths, images, extrinsics, intrinsics, adapter)
        return decoder(g, tgt_extrinsics, tgt_intrinsics, near, far, image_shape).color
    B, V, HW, C = head.shape
    b, v = tgt_extrinsics.shape[:2]
    Ht, Wt = image_shape
    acams = adapter_cameras(extrinsics, intrinsics, adapter.cfg.sh_degree)
    view_scene = [i // v for i in range(b * v)]
    tcams = raster.camera_inputs(tgt_extrinsics.reshape(b * v, 4, 4), tgt_intrinsics.reshape(b * v, 3, 3),
                                 near.reshape(b * v), far.reshape(b * v), decoder.background_color.expand(b * v, 3),
                                 view_scene, True)
    color = _HeadRender.apply(head.contiguous().float(), depths.reshape(B, V, HW).contiguous().float(),
                              images.detach().contiguous().float(), acams, adapter.cfg.gaussian_scale_min,
                              adapter.cfg.gaussian_scale_max, adapter.sh_mask.to(head.device).float().contiguous(),
                              adapter.d_sh, tcams, view_scene, Ht, Wt, decoder.raster_ctx)
    return color.reshape(b, v, 3, Ht, Wt)
