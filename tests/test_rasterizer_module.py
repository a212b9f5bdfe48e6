"""The drop-in boundary itself: `GaussianRasterizer(settings)(...)` (the module the reference
calls at src/model/decoder/cuda_splatting.py:98-123), render_depth_cuda (:225-264),
render_cuda_orthographic (:129-219) and the decoder's depth_mode (decoder_splatting_cuda.py:
69-91), driven with the settings and tensors the REFERENCE wrapper handed to its rasterizer
(tests/golden/cuda_splatting_settings.npz, recorded by tests/golden/make_golden.py) and
checked against the oracle fed the same recorded inputs.

The argument-contract tests (exactly one of shs / colors_precomp, one of scales+rotations /
cov3D_precomp) raise before any device work and run on CPU.
"""
from __future__ import annotations

import math
from pathlib import Path

import numpy as np
import pytest
import torch

GOLD = Path(__file__).parent / "golden" / "cuda_splatting_settings.npz"
L1_BAR = 1e-4


def _gold():
    return np.load(GOLD)


def _settings(Gd, tag, i, dev, bg=None, scale_modifier=1.0):
    from my_depthsplat_amd.rasterizer import GaussianRasterizationSettings
    H, W = (int(x) for x in Gd["image_hw"])
    t = lambda a: torch.from_numpy(np.asarray(a, np.float32)).to(dev)  # noqa: E731
    tan = Gd[f"si_view{i}_tanfov"] if f"{tag}_view{i}_tanfov" not in Gd.files else Gd[f"{tag}_view{i}_tanfov"]
    if bg is None:
        bg = Gd[f"si_view{i}_bg"]
    return GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=float(tan[0]), tanfovy=float(tan[1]), bg=t(bg),
        scale_modifier=scale_modifier, viewmatrix=t(Gd[f"{tag}_view{i}_viewmatrix"]),
        projmatrix=t(Gd[f"{tag}_view{i}_projmatrix"]), sh_degree=int(Gd["si_view0_shdeg"]),
        campos=t(Gd[f"{tag}_view{i}_campos"]), prefiltered=False, debug=False)


def _oracle(Gd, tag, i, means, shs, colors, opac, cov6, bg):
    from oracle import raster as orc
    H, W = (int(x) for x in Gd["image_hw"])
    tan = Gd[f"si_view{i}_tanfov"] if f"{tag}_view{i}_tanfov" not in Gd.files else Gd[f"{tag}_view{i}_tanfov"]
    deg = int(Gd["si_view0_shdeg"]) if shs is not None else 0
    return orc.View(means, shs, colors, opac, cov6, Gd[f"{tag}_view{i}_viewmatrix"], Gd[f"{tag}_view{i}_projmatrix"],
                    Gd[f"{tag}_view{i}_campos"], float(tan[0]), float(tan[1]), np.asarray(bg, np.float32), H, W, deg)


def _close(hip, ref, what, rel=5e-4):
    err = float(np.abs(hip - ref).max() / (np.abs(ref).max() + 1e-12))
    assert err < rel, (what, err)


# ---------------------------------------------------------------- argument contract (CPU)

def _module_cpu():
    from my_depthsplat_amd.rasterizer import GaussianRasterizationSettings, GaussianRasterizer
    s = GaussianRasterizationSettings(8, 8, 0.5, 0.5, torch.zeros(3), 1.0, torch.eye(4), torch.eye(4), 0,
                                      torch.zeros(3), False, False)
    return GaussianRasterizer(s)


@pytest.mark.parametrize("case", ["both_colors", "no_colors", "both_cov", "no_cov", "half_scale_rot"])
def test_argument_contract_raises(case):
    """The upstream module's two exception cases (one of shs / colors_precomp; one of the
    scales+rotations pair / cov3D_precomp), raised before any device work."""
    r = _module_cpu()
    P = 4
    m, m2, o = torch.zeros(P, 3), torch.zeros(P, 3), torch.ones(P, 1)
    shs, col, cov = torch.zeros(P, 1, 3), torch.zeros(P, 3), torch.zeros(P, 6)
    sc, rot = torch.ones(P, 3), torch.tensor([[1.0, 0, 0, 0]]).repeat(P, 1)
    kw = {"both_colors": dict(shs=shs, colors_precomp=col, cov3D_precomp=cov),
          "no_colors": dict(cov3D_precomp=cov),
          "both_cov": dict(shs=shs, scales=sc, rotations=rot, cov3D_precomp=cov),
          "no_cov": dict(shs=shs),
          "half_scale_rot": dict(shs=shs, scales=sc)}[case]
    with pytest.raises(Exception, match="exactly one|excatly one"):
        r(m, m2, o, **kw)


def test_scale_rotation_covariance_matches_upstream_formula():
    """cov6_from_scale_rotation = upstream computeCov3D: Sigma = R S S^T R^T, S = diag(mod *
    scale), R from the (r, x, y, z) quaternion as given; stored (xx, xy, xz, yy, yz, zz)."""
    from my_depthsplat_amd.rasterizer import cov6_from_scale_rotation
    g = torch.Generator().manual_seed(0)
    s = torch.rand(16, 3, generator=g, dtype=torch.float64) + 0.1
    q = torch.randn(16, 4, generator=g, dtype=torch.float64)
    q = q / q.norm(dim=-1, keepdim=True)
    got = cov6_from_scale_rotation(s, q, 0.7).numpy()
    for k in range(16):
        r, x, y, z = q[k].tolist()
        R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)],
                      [2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)],
                      [2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)]])
        Sg = R @ np.diag((0.7 * s[k].numpy()) ** 2) @ R.T
        np.testing.assert_allclose(got[k], Sg[[0, 0, 0, 1, 1, 2], [0, 1, 2, 1, 2, 2]], rtol=1e-12, atol=1e-14)


# ---------------------------------------------------------------- module on the device

@pytest.mark.gpu
@pytest.mark.parametrize("i", [0, 1, 2])
def test_module_shs_cov3d_forward_backward(gpu, i):
    """GaussianRasterizer with the recorded scale-invariant settings of view i, shs +
    cov3D_precomp (the reference's call): image, radii and the gradients of means3D,
    means2D, shs, opacities and cov3D_precomp vs the oracle."""
    from my_depthsplat_amd.rasterizer import GaussianRasterizer
    Gd = _gold()
    H, W = (int(x) for x in Gd["image_hw"])
    arr = {k: Gd[f"si_view{i}_{k}"] for k in ("means3D", "shs", "opacities", "cov3D_precomp")}
    t = {k: torch.from_numpy(v).to(gpu).requires_grad_(True) for k, v in arr.items()}
    means2D = torch.zeros_like(t["means3D"], requires_grad=True)
    r = GaussianRasterizer(_settings(Gd, "si", i, gpu))
    image, radii = r(means3D=t["means3D"], means2D=means2D, shs=t["shs"], colors_precomp=None,
                     opacities=t["opacities"], scales=None, rotations=None, cov3D_precomp=t["cov3D_precomp"])
    assert image.shape == (3, H, W) and radii.shape == (arr["means3D"].shape[0],) and radii.dtype == torch.int32
    dpix = torch.randn(3, H, W, generator=torch.Generator().manual_seed(i))
    (image * dpix.to(gpu)).sum().backward()
    torch.cuda.synchronize()
    o = _oracle(Gd, "si", i, arr["means3D"], arr["shs"], None, arr["opacities"], arr["cov3D_precomp"],
                Gd[f"si_view{i}_bg"])
    oc, _, _ = o.image()
    assert float(np.abs(image.detach().cpu().numpy() - oc).mean()) < L1_BAR
    np.testing.assert_array_equal(radii.cpu().numpy(), o.geom()["radii"])
    gr = o.backward(dpix.numpy(), f64=True)
    _close(means2D.grad.cpu().numpy(), gr["dmean2D"], "means2D")
    _close(t["means3D"].grad.cpu().numpy(), gr["dmean3D"], "means3D")
    _close(t["shs"].grad.cpu().numpy(), gr["dsh"], "shs")
    _close(t["opacities"].grad.cpu().numpy().reshape(-1), gr["dopacity"], "opacities")
    _close(t["cov3D_precomp"].grad.cpu().numpy(), gr["dcov6"], "cov3D")
    o.close()


@pytest.mark.gpu
@pytest.mark.parametrize("i", [0, 2])
def test_module_colors_precomp(gpu, i):
    """colors_precomp path with the recorded non-scale-invariant settings (use_sh=False call)."""
    from my_depthsplat_amd.rasterizer import GaussianRasterizer
    Gd = _gold()
    arr = {k: Gd[f"ns_view{i}_{k}"] for k in ("means3D", "colors_precomp", "cov3D_precomp")}
    opac = Gd[f"si_view{i}_opacities"]
    t = {k: torch.from_numpy(v).to(gpu).requires_grad_(True) for k, v in arr.items()}
    op = torch.from_numpy(opac).to(gpu)
    r = GaussianRasterizer(_settings(Gd, "ns", i, gpu))
    image, _ = r(t["means3D"], torch.zeros_like(t["means3D"]), op, colors_precomp=t["colors_precomp"],
                 cov3D_precomp=t["cov3D_precomp"])
    dpix = torch.randn(image.shape, generator=torch.Generator().manual_seed(10 + i))
    (image * dpix.to(gpu)).sum().backward()
    torch.cuda.synchronize()
    o = _oracle(Gd, "ns", i, arr["means3D"], None, arr["colors_precomp"], opac, arr["cov3D_precomp"],
                Gd[f"si_view{i}_bg"])
    oc, _, _ = o.image()
    assert float(np.abs(image.detach().cpu().numpy() - oc).mean()) < L1_BAR
    gr = o.backward(dpix.numpy(), f64=True)
    _close(t["colors_precomp"].grad.cpu().numpy(), gr["dcolor"], "colors_precomp")
    _close(t["means3D"].grad.cpu().numpy(), gr["dmean3D"], "means3D")
    o.close()


@pytest.mark.gpu
def test_module_scales_rotations_scale_modifier(gpu):
    """scales + rotations + scale_modifier (no cov3D_precomp): the covariance is built as the
    upstream computeCov3D does; the oracle gets the float64-built cov6. Gradients reach
    scales and rotations through it (checked against the oracle's dcov6 chained in float64)."""
    from my_depthsplat_amd.rasterizer import GaussianRasterizer
    Gd = _gold()
    i, mod = 1, 0.8
    means = Gd[f"si_view{i}_means3D"]
    P = means.shape[0]
    g = torch.Generator().manual_seed(4)
    scales = (torch.rand(P, 3, generator=g) * 0.08 + 0.02).numpy()
    rots = torch.randn(P, 4, generator=g)
    rots = (rots / rots.norm(dim=-1, keepdim=True)).numpy()
    t_s = torch.from_numpy(scales).to(gpu).requires_grad_(True)
    t_r = torch.from_numpy(rots).to(gpu).requires_grad_(True)
    m = torch.from_numpy(means).to(gpu)
    r = GaussianRasterizer(_settings(Gd, "si", i, gpu, scale_modifier=mod))
    image, _ = r(m, torch.zeros_like(m), torch.from_numpy(Gd[f"si_view{i}_opacities"]).to(gpu),
                 shs=torch.from_numpy(Gd[f"si_view{i}_shs"]).to(gpu), scales=t_s, rotations=t_r)
    dpix = torch.randn(image.shape, generator=torch.Generator().manual_seed(5))
    (image * dpix.to(gpu)).sum().backward()
    torch.cuda.synchronize()
    # float64 reference covariance, and its vector-Jacobian product for the oracle's dcov6
    s64 = torch.from_numpy(scales).double().requires_grad_(True)
    q64 = torch.from_numpy(rots).double().requires_grad_(True)
    from my_depthsplat_amd.rasterizer import cov6_from_scale_rotation
    c64 = cov6_from_scale_rotation(s64, q64, mod)
    o = _oracle(Gd, "si", i, means, Gd[f"si_view{i}_shs"], None, Gd[f"si_view{i}_opacities"],
                c64.detach().float().numpy(), Gd[f"si_view{i}_bg"])
    oc, _, _ = o.image()
    assert float(np.abs(image.detach().cpu().numpy() - oc).mean()) < L1_BAR
    gr = o.backward(dpix.numpy(), f64=True)
    (c64 * torch.from_numpy(gr["dcov6"]).double()).sum().backward()
    _close(t_s.grad.cpu().numpy(), s64.grad.numpy(), "scales", rel=5e-3)
    _close(t_r.grad.cpu().numpy(), q64.grad.numpy(), "rotations", rel=5e-3)
    o.close()


# ---------------------------------------------------------------- depth / orthographic renders

def _tensors(Gd, dev, b=None):
    sl = slice(None) if b is None else slice(b, b + 1)
    return {k: torch.from_numpy(Gd[k][sl]).to(dev) for k in ("extrinsics", "intrinsics", "near", "far", "bg", "means",
                                                              "cov", "sh", "opacities")}


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["depth", "disparity", "log"])
def test_render_depth_cuda_vs_oracle(gpu, mode):
    """render_depth_cuda (3 modes) vs the oracle fed the colours, means and settings the
    reference wrapper recorded for that mode (bg = 0; output = channel mean)."""
    from my_depthsplat_amd.cuda_splatting import render_depth_cuda
    Gd = _gold()
    H, W = (int(x) for x in Gd["image_hw"])
    t = _tensors(Gd, gpu)
    out = render_depth_cuda(t["extrinsics"], t["intrinsics"], t["near"], t["far"], (H, W), t["means"], t["cov"],
                            t["opacities"], mode=mode).cpu().numpy()
    assert out.shape == (3, H, W)
    for i in range(3):
        o = _oracle(Gd, "si", i, Gd[f"depth_{mode}_view{i}_means3D"], None, Gd[f"depth_{mode}_view{i}_colors_precomp"],
                    Gd[f"si_view{i}_opacities"], Gd[f"si_view{i}_cov3D_precomp"], np.zeros(3, np.float32))
        oc, _, _ = o.image()
        ref = oc.mean(axis=0)
        scale = float(np.abs(ref).mean()) + 1e-6
        assert float(np.abs(out[i] - ref).mean()) < L1_BAR * scale, (mode, i)
        o.close()


@pytest.mark.gpu
def test_decoder_depth_mode_vs_oracle(gpu):
    """DecoderSplattingCUDA(..., depth_mode='depth'): colour and depth outputs for one scene
    seen from the 3 recorded cameras vs the oracle (camera settings and depth colours from
    the fixture-pinned restatements camera_settings / depth_colors)."""
    from my_depthsplat_amd.cuda_splatting import _cov6, camera_settings, depth_colors
    from my_depthsplat_amd.decoder import DecoderSplattingCUDA, DecoderSplattingCUDACfg, Gaussians
    from oracle import raster as orc
    Gd = _gold()
    H, W = (int(x) for x in Gd["image_hw"])
    c = {k: torch.from_numpy(Gd[k]) for k in ("extrinsics", "intrinsics", "near", "far", "means", "cov", "sh",
                                               "opacities")}
    gs = Gaussians(c["means"][:1].to(gpu), c["cov"][:1].to(gpu), c["sh"][:1].to(gpu), c["opacities"][:1].to(gpu))
    dec = DecoderSplattingCUDA(DecoderSplattingCUDACfg("splatting_cuda"), {"background_color": [0.1, 0.2, 0.3]}).to(gpu)
    out = dec(gs, c["extrinsics"][None].to(gpu), c["intrinsics"][None].to(gpu), c["near"][None].to(gpu),
              c["far"][None].to(gpu), (H, W), depth_mode="depth")
    assert out.color.shape == (1, 3, 3, H, W) and out.depth.shape == (1, 3, H, W)
    st = {k: v.numpy() for k, v in camera_settings(c["extrinsics"], c["intrinsics"], c["near"], c["far"]).items()}
    means0 = c["means"][0].numpy()
    shs0 = c["sh"][0].transpose(-1, -2).contiguous().numpy()
    cov60 = _cov6(c["cov"][0]).contiguous().numpy()
    op0 = c["opacities"][0].numpy()
    fake = depth_colors(c["extrinsics"], c["means"][:1].expand(3, -1, -1), c["near"], c["far"], "depth").numpy()
    for i in range(3):
        o = orc.render_settings(means0, shs0, None, op0, cov60, st, i, np.array([0.1, 0.2, 0.3], np.float32), H, W, 2)
        oc, _, _ = o.image()
        assert float(np.abs(out.color[0, i].cpu().numpy() - oc).mean()) < L1_BAR
        o.close()
        col = np.repeat(fake[i][:, None], 3, axis=1).astype(np.float32)
        o = orc.render_settings(means0, None, col, op0, cov60, st, i, np.zeros(3, np.float32), H, W, 0)
        od, _, _ = o.image()
        ref = od.mean(axis=0)
        assert float(np.abs(out.depth[0, i].cpu().numpy() - ref).mean()) < L1_BAR * (float(np.abs(ref).mean()) + 1e-6)
        o.close()


@pytest.mark.gpu
def test_render_cuda_orthographic_vs_oracle(gpu):
    """render_cuda_orthographic (fov 10 deg, the caller's value) vs the oracle fed the
    pseudo-orthographic settings the reference wrapper recorded."""
    from my_depthsplat_amd.cuda_splatting import _cov6, render_cuda_orthographic
    Gd = _gold()
    H, W = (int(x) for x in Gd["image_hw"])
    t = _tensors(Gd, gpu, b=0)
    out = render_cuda_orthographic(t["extrinsics"], torch.from_numpy(Gd["ortho_width"]).to(gpu),
                                   torch.from_numpy(Gd["ortho_height"]).to(gpu), t["near"], t["far"], (H, W), t["bg"],
                                   t["means"], t["cov"], t["sh"], t["opacities"], fov_degrees=10.0)
    torch.cuda.synchronize()
    shs = torch.from_numpy(Gd["sh"][0]).transpose(-1, -2).contiguous().numpy()
    cov6 = _cov6(torch.from_numpy(Gd["cov"][0])).contiguous().numpy()
    o = _oracle(Gd, "ortho", 0, Gd["means"][0], shs, None, Gd["opacities"][0], cov6, Gd["bg"][0])
    oc, _, _ = o.image()
    assert out.shape == (1, 3, H, W)
    assert float(np.abs(out[0].cpu().numpy() - oc).mean()) < L1_BAR
    assert float(np.abs(oc).sum()) > 0
    o.close()
    assert math.isfinite(float(out.sum()))
