"""Fused HIP Gaussian adapter (dga_adapter_fwd/bwd) vs the torch composition of the
reference modules (gaussians_from_head_torch: GaussianAdapter + rotate_sh + encoder glue,
itself pinned to the reference by tests/golden/adapter.npz). fp32 reference, same device."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _random_c2w(n, g):
    q = torch.randn(n, 4, generator=g)
    q = q / q.norm(dim=-1, keepdim=True)
    i, j, k, r = q.unbind(-1)
    R = torch.stack([1 - 2 * (j * j + k * k), 2 * (i * j - k * r), 2 * (i * k + j * r),
                     2 * (i * j + k * r), 1 - 2 * (i * i + k * k), 2 * (j * k - i * r),
                     2 * (i * k - j * r), 2 * (j * k + i * r), 1 - 2 * (i * i + j * j)], -1).reshape(n, 3, 3)
    m = torch.eye(4).repeat(n, 1, 1)
    m[:, :3, :3] = R
    m[:, :3, 3] = torch.randn(n, 3, generator=g)
    return m


def _inputs(sh_degree, B=2, V=2, H=8, W=12, seed=0, dev="cuda"):
    from my_depthsplat_amd.gaussian_adapter import GaussianAdapter, GaussianAdapterCfg
    g = torch.Generator().manual_seed(seed)
    adapter = GaussianAdapter(GaussianAdapterCfg(1e-10, 3.0, sh_degree))
    C = 3 + adapter.d_in
    head = torch.randn(B, V, H * W, C, generator=g)
    head[0, 0, :5, 3:6] = 30.0   # softplus above the torch threshold and clamped at scale_max
    head[0, 1, :3, 3:6] = -40.0  # clamped at scale_min
    depths = torch.rand(B, V, H * W, 1, 1, generator=g) * 9 + 1
    images = torch.rand(B, V, 3, H, W, generator=g)
    ext = _random_c2w(B * V, g).reshape(B, V, 4, 4)
    K = torch.tensor([[1.1, 0.0, 0.52], [0.0, 0.9, 0.47], [0, 0, 1]]).expand(B, V, 3, 3).clone()
    to = lambda t: t.to(dev)  # noqa: E731
    return to(head), to(depths), to(images), to(ext), to(K), adapter.to(dev)


# (8, 12): views split across workgroups (per-lane camera reads); (16, 32): every 256-row
# workgroup inside one view (the workgroup-uniform camera path, dga_adapter.hip UNI)
SIZES = [(8, 12), (16, 32)]


@pytest.mark.parametrize("sh_degree", [0, 1, 2, 3])
@pytest.mark.parametrize("H,W", SIZES)
def test_fused_adapter_forward_matches_torch(gpu, sh_degree, H, W):
    from my_depthsplat_amd.adapter_hip import fused_gaussians_from_head
    from my_depthsplat_amd.gaussian_adapter import gaussians_from_head_torch
    head, depths, images, ext, K, adapter = _inputs(sh_degree, H=H, W=W, seed=sh_degree)
    a = fused_gaussians_from_head(head, depths, images, ext, K, adapter)
    b = gaussians_from_head_torch(head, depths, images, ext, K, adapter)
    for name in ("means", "covariances", "harmonics", "opacities"):
        x, y = getattr(a, name), getattr(b, name)
        assert x.shape == y.shape, name
        torch.testing.assert_close(x, y, rtol=2e-5, atol=2e-5, msg=name)


@pytest.mark.parametrize("sh_degree", [1, 2, 3])
@pytest.mark.parametrize("H,W", SIZES)
def test_fused_adapter_backward_matches_autograd(gpu, sh_degree, H, W):
    from my_depthsplat_amd.adapter_hip import fused_gaussians_from_head
    from my_depthsplat_amd.gaussian_adapter import gaussians_from_head_torch
    head, depths, images, ext, K, adapter = _inputs(sh_degree, H=H, W=W, seed=10 + sh_degree)
    gen = torch.Generator(device=head.device).manual_seed(3)
    outs = []
    for fn in (fused_gaussians_from_head, gaussians_from_head_torch):
        h = head.clone().requires_grad_(True)
        d = depths.clone().requires_grad_(True)
        gs = fn(h, d, images, ext, K, adapter)
        outs.append((h, d, gs))
    # same random cotangents for both (full 3x3 covariance gradient, like an arbitrary consumer)
    cot = [torch.randn(t.shape, generator=gen, device=head.device) for t in
           (outs[0][2].means, outs[0][2].covariances, outs[0][2].harmonics, outs[0][2].opacities)]
    grads = []
    for h, d, gs in outs:
        loss = sum((t * c).sum() for t, c in zip((gs.means, gs.covariances, gs.harmonics, gs.opacities), cot))
        loss.backward()
        grads.append((h.grad, d.grad))
    (h1, d1), (h2, d2) = grads
    scale = h2.abs().max()
    torch.testing.assert_close(h1, h2, rtol=1e-4, atol=1e-5 * float(scale), msg="dhead")
    torch.testing.assert_close(d1, d2, rtol=1e-4, atol=1e-5, msg="ddepth")


def test_fused_adapter_drives_the_decoder(gpu):
    """gaussians_from_head on device tensors takes the fused path and feeds the rasterizer."""
    from my_depthsplat_amd.decoder import DecoderSplattingCUDA, DecoderSplattingCUDACfg
    from my_depthsplat_amd.gaussian_adapter import gaussians_from_head, gaussians_from_head_torch
    from my_depthsplat_amd.synthetic import context_cameras, target_cameras
    head, depths, images, _, K, adapter = _inputs(2, B=1, V=2, H=32, W=32, seed=5)
    ext = context_cameras(2)[None].to(head.device)
    tgt = target_cameras(context_cameras(2), 2)[None].to(head.device)
    Kt = K[:, :1].expand(1, 2, 3, 3).contiguous()
    dec = DecoderSplattingCUDA(DecoderSplattingCUDACfg("splatting_cuda"), {"background_color": [0, 0, 0]}).to(head.device)
    near = torch.full((1, 2), 0.5, device=head.device)
    far = torch.full((1, 2), 100.0, device=head.device)
    a = dec(gaussians_from_head(head, depths, images, ext, K, adapter), tgt, Kt, near, far, (32, 32)).color
    b = dec(gaussians_from_head_torch(head, depths, images, ext, K, adapter), tgt, Kt, near, far, (32, 32)).color
    assert float((a - b).abs().mean()) < 1e-5
    assert math.isfinite(float(a.sum()))


def test_device_camera_blocks_match_torch(gpu):
    """dga_adapter_cameras (K^-1 and Wigner-D on the device) vs the torch construction."""
    from my_depthsplat_amd.adapter_hip import adapter_cameras, adapter_cameras_torch
    _, _, _, ext, K, _ = _inputs(3, B=3, V=2, seed=21)
    for deg in (0, 1, 2, 3):
        a = adapter_cameras(ext, K, deg)
        b = adapter_cameras_torch(ext, K, deg)
        torch.testing.assert_close(a, b, rtol=1e-5, atol=2e-6)


def test_reference_signature_forward_vs_golden(gpu):
    """GaussianAdapter.forward (reference signature, gaussian_adapter.py:49-102) on device
    tensors runs dga_adapter_forward; checked against the outputs the REFERENCE module
    produced for the same inputs (tests/golden/adapter.npz, identity c2w rotations)."""
    from pathlib import Path

    import numpy as np

    from my_depthsplat_amd.gaussian_adapter import GaussianAdapter, GaussianAdapterCfg
    G = np.load(Path(__file__).parent / "golden" / "adapter.npz")
    T = lambda k: torch.from_numpy(G[k]).to(gpu)  # noqa: E731
    ad = GaussianAdapter(GaussianAdapterCfg(1e-10, 3.0, 2)).to(gpu)
    h, w = G["images"].shape[-2:]
    out = ad(T("extrinsics")[:, :, None, None, None], T("intrinsics")[:, :, None, None, None], T("coordinates"),
             T("depths"), T("opacities"), T("raw"), (h, w), input_images=T("images"))
    for name, key, rtol, atol in (("means", "means", 1e-5, 1e-5), ("covariances", "covariances", 1e-5, 1e-7),
                                  ("harmonics", "harmonics", 1e-5, 1e-6), ("scales", "scales", 1e-6, 1e-6),
                                  ("rotations", "rotations", 1e-6, 1e-6), ("opacities", "out_opacities", 0, 0)):
        got = getattr(out, name).cpu().numpy()
        assert got.shape == G[key].shape, name
        np.testing.assert_allclose(got, G[key], rtol=rtol, atol=atol, err_msg=name)


@pytest.mark.parametrize("sh_degree,srf", [(2, 1), (3, 2), (0, 1)])
def test_reference_signature_matches_torch_fwd_bwd(gpu, sh_degree, srf):
    """dga_adapter_forward/backward vs the torch composition (forward_torch) on random
    rotations, with `srf` surfaces per pixel: outputs within 2e-5, gradients of
    raw_gaussians, coordinates and depths (cotangents on every output incl. scales and
    rotations) within 1e-4."""
    from my_depthsplat_amd.projection import sample_image_grid
    head, depths, images, ext, K, adapter = _inputs(sh_degree, B=2, V=2, H=8, W=12, seed=40 + sh_degree)
    B, V, HW = head.shape[:3]
    g = torch.Generator(device=gpu).manual_seed(9)
    raw = torch.randn(B, V, HW, srf, 1, adapter.d_in, generator=g, device=gpu)
    raw[0, 0, :4, 0, 0, :3] = 30.0  # scale clamped at the max (and softplus past its threshold)
    xy, _ = sample_image_grid((8, 12), gpu)
    coords = xy.reshape(1, 1, HW, 1, 1, 2) + 0.01 * torch.randn(B, V, HW, srf, 1, 2, generator=g, device=gpu)
    dep = torch.rand(B, V, HW, srf, 1, generator=g, device=gpu) * 9 + 1
    opac = torch.rand(B, V, HW, srf, 1, generator=g, device=gpu)
    e, k = ext[:, :, None, None, None], K[:, :, None, None, None]
    res = []
    for fn in (adapter.forward, adapter.forward_torch):
        r_ = raw.clone().requires_grad_(True)
        c_ = coords.clone().requires_grad_(True)
        d_ = dep.clone().requires_grad_(True)
        out = fn(e, k, c_, d_, opac, r_, (8, 12), input_images=images)
        res.append((r_, c_, d_, out))
    names = ("means", "covariances", "harmonics", "scales", "rotations")
    for name in names:
        torch.testing.assert_close(getattr(res[0][3], name), getattr(res[1][3], name), rtol=2e-5, atol=2e-5,
                                   msg=name)
    assert res[0][3].opacities is opac
    cot = [torch.randn(getattr(res[0][3], n).shape, generator=g, device=gpu) for n in names]
    grads = []
    for r_, c_, d_, out in res:
        sum((getattr(out, n) * c).sum() for n, c in zip(names, cot)).backward()
        grads.append((r_.grad, c_.grad, d_.grad))
    for a, b, name in zip(grads[0], grads[1], ("raw", "coordinates", "depths")):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5 * float(b.abs().max()), msg=name)


def test_reference_signature_camera_grads_and_broadcast(gpu):
    """Cameras that require grad (pose refinement) get gradients as in the reference: the
    module routes them to the torch composition on the device instead of silently detaching
    them. Cameras broadcast over the batch ([1, v, ...]) are expanded for the fused kernel."""
    from my_depthsplat_amd.projection import sample_image_grid
    head, depths, images, ext, K, adapter = _inputs(2, B=2, V=2, H=8, W=12, seed=77)
    B, V, HW = head.shape[:3]
    g = torch.Generator(device=gpu).manual_seed(3)
    raw = torch.randn(B, V, HW, 1, 1, adapter.d_in, generator=g, device=gpu)
    xy, _ = sample_image_grid((8, 12), gpu)
    coords = xy.reshape(1, 1, HW, 1, 1, 2).expand(B, V, HW, 1, 1, 2)
    dep = torch.rand(B, V, HW, 1, 1, generator=g, device=gpu) * 9 + 1
    opac = torch.rand(B, V, HW, 1, 1, generator=g, device=gpu)
    e = ext[:, :, None, None, None].clone().requires_grad_(True)
    k = K[:, :, None, None, None]
    out = adapter(e, k, coords, dep, opac, raw, (8, 12), input_images=images)
    out.means.sum().backward()
    assert e.grad is not None and float(e.grad.abs().max()) > 0
    e2 = ext[:, :, None, None, None].detach().clone().requires_grad_(True)
    adapter.forward_torch(e2, k, coords, dep, opac, raw, (8, 12), input_images=images).means.sum().backward()
    torch.testing.assert_close(e.grad, e2.grad)
    # one camera block per view shared by the batch: broadcast like the reference
    e1 = ext[:1, :, None, None, None]
    a = adapter(e1, k, coords, dep, opac, raw, (8, 12), input_images=images)
    b = adapter.forward_torch(e1, k, coords, dep, opac, raw, (8, 12), input_images=images)
    torch.testing.assert_close(a.means, b.means, rtol=2e-5, atol=2e-5)
    torch.testing.assert_close(a.harmonics, b.harmonics, rtol=2e-5, atol=2e-5)


@pytest.mark.parametrize("BV,C,r,h,w", [(3, 37, 8, 7, 12), (2, 5, 1, 9, 33), (1, 38, 4, 5, 20)])
def test_head_rows_matches_torch_permute(gpu, BV, C, r, h, w):
    """dga_head_rows (the head glue's pixel shuffle + "(b v) c h w -> b v (h w) c" in one
    LDS-tiled pass, encoder_depthsplat.py:224-233 at r = 1) and its backward: bit-identical to
    the torch permutation and to its autograd gradient, on tiles that do not divide w."""
    from my_depthsplat_amd.training import head_rows
    gen = torch.Generator().manual_seed(BV * 100 + C)
    x = torch.randn(BV, C * r * r, h, w, generator=gen).to(gpu).requires_grad_(True)
    rows = head_rows(x, C, r)
    x_ref = x.detach().clone().requires_grad_(True)
    ref = x_ref.view(BV, C, r, r, h, w).permute(0, 4, 2, 5, 3, 1).reshape(BV, h * r * w * r, C)
    torch.cuda.synchronize()
    assert rows.shape == ref.shape and torch.equal(rows, ref)
    g = torch.randn(rows.shape, generator=gen).to(gpu)
    rows.backward(g)
    ref.backward(g)
    torch.cuda.synchronize()
    assert torch.equal(x.grad, x_ref.grad)
