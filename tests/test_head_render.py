"""Fused adapter + rasterizer training node (my_depthsplat_amd/head_render.py, dsr_head_bwd):
the colour and the head / depth gradients must equal the two-module composition
(gaussians_from_head -> DecoderSplattingCUDA) bit for bit — the same kernels up to the
rasterizer's K7 and the same float operations after it (dga_math.h, pbwd_views)."""
import pytest
import torch

from test_adapter_gpu import _inputs


def _targets(B, v, dev, seed=3):
    from my_depthsplat_amd.synthetic import context_cameras, target_cameras
    tgt = target_cameras(context_cameras(2), v)[None].repeat(B, 1, 1, 1).to(dev)
    K = torch.tensor([[1.0, 0, 0.5], [0, 1.0, 0.5], [0, 0, 1]], device=dev).expand(B, v, 3, 3).contiguous()
    near = torch.full((B, v), 0.5, device=dev)
    far = torch.full((B, v), 100.0, device=dev)
    return tgt, K, near, far


def _context(B, V, H, W, sh_degree, dev, seed):
    from my_depthsplat_amd.synthetic import context_cameras
    head, depths, images, _, _, adapter = _inputs(sh_degree, B=B, V=V, H=H, W=W, seed=seed, dev=dev)
    ext = context_cameras(V)[None].repeat(B, 1, 1, 1).to(dev)
    K = torch.tensor([[1.0, 0, 0.5], [0, 1.0, 0.5], [0, 0, 1]], device=dev).expand(B, V, 3, 3).contiguous()
    return head, depths, images, ext, K, adapter


@pytest.mark.gpu
@pytest.mark.parametrize("sh_degree,H,W", [(2, 64, 64), (1, 32, 64), (2, 24, 40)])
def test_head_render_matches_two_module_path(gpu, sh_degree, H, W):
    """(64, 64) / (32, 64): the fused node (H*W % 256 == 0); (24, 40): H*W = 960, the composed
    fallback. Colour, dhead and ddepth bit-identical to the composition's."""
    from my_depthsplat_amd.decoder import DecoderSplattingCUDA, DecoderSplattingCUDACfg
    from my_depthsplat_amd.gaussian_adapter import gaussians_from_head
    from my_depthsplat_amd.head_render import fusable, render_from_head
    B, V, v = 2, 2, 3
    head, depths, images, ext, K, adapter = _context(B, V, H, W, sh_degree, gpu, seed=7)
    tgt, tK, near, far = _targets(B, v, gpu)
    assert fusable(head, images, adapter) == (H * W % 256 == 0)
    dcolor = torch.randn(B, v, 3, H, W, generator=torch.Generator().manual_seed(5)).to(gpu)
    outs = []
    for fused in (True, False):
        dec = DecoderSplattingCUDA(DecoderSplattingCUDACfg("splatting_cuda"), {"background_color": [0.0, 0.0, 0.0]}).to(gpu)
        hd = head.clone().requires_grad_(True)
        dp = depths.clone().requires_grad_(True)
        if fused:
            color = render_from_head(dec, hd, dp, images, ext, K, adapter, tgt, tK, near, far, (H, W))
        else:
            g = gaussians_from_head(hd, dp, images, ext, K, adapter)
            color = dec(g, tgt, tK, near, far, (H, W)).color
        (color * dcolor).sum().backward()
        outs.append((color.detach(), hd.grad, dp.grad))
    for a, b, name in zip(outs[0], outs[1], ("color", "dhead", "ddepth")):
        assert a.shape == b.shape, name
        assert torch.equal(a, b), f"{name}: max |diff| {float((a - b).abs().max())}"
    assert outs[0][1].abs().max() > 0


@pytest.mark.gpu
def test_head_render_backward_is_deterministic(gpu):
    from my_depthsplat_amd.decoder import DecoderSplattingCUDA, DecoderSplattingCUDACfg
    from my_depthsplat_amd.head_render import render_from_head
    B, V, v, H, W = 2, 2, 4, 64, 64
    head, depths, images, ext, K, adapter = _context(B, V, H, W, 2, gpu, seed=9)
    tgt, tK, near, far = _targets(B, v, gpu)
    dec = DecoderSplattingCUDA(DecoderSplattingCUDACfg("splatting_cuda"), {"background_color": [0.0, 0.0, 0.0]}).to(gpu)
    grads = []
    for _ in range(2):
        hd = head.clone().requires_grad_(True)
        render_from_head(dec, hd, depths, images, ext, K, adapter, tgt, tK, near, far, (H, W)).square().sum().backward()
        grads.append(hd.grad)
    assert torch.equal(grads[0], grads[1])


def test_head_render_fallback_rules_without_gpu():
    """The fused node needs device tensors and H*W % 256 == 0; anything else composes the two
    modules (host tensors never reach the HIP library)."""
    from my_depthsplat_amd.gaussian_adapter import GaussianAdapter, GaussianAdapterCfg
    from my_depthsplat_amd.head_render import fusable
    ad = GaussianAdapter(GaussianAdapterCfg(1e-10, 3.0, 2))
    assert not fusable(torch.zeros(1, 2, 4096, 3 + ad.d_in), torch.zeros(1, 2, 3, 64, 64), ad)
