"""Pinning the CPU rasterizer restatement (oracle/dsr_oracle.cpp), which the HIP kernels
are checked against. The upstream CUDA rasterizer is absent (parity unpinned), so the
oracle is pinned here by analytic known-answer cases and by torch.autograd of a dense
differentiable restatement (tests/dense_raster.py) for the backward."""
from __future__ import annotations

import math

import numpy as np
import pytest
import torch

import dense_raster
from my_depthsplat_amd.cuda_splatting import camera_settings
from oracle import raster as orc


def cam(H, W, fx=1.0, fy=1.0, near=0.5, far=100.0, c2w=None, scale_invariant=False):
    c2w = torch.eye(4) if c2w is None else c2w
    K = torch.tensor([[fx, 0, 0.5], [0, fy, 0.5], [0, 0, 1.0]])
    st = camera_settings(c2w[None], K[None], torch.tensor([near]), torch.tensor([far]), scale_invariant)
    return {k: v[0].numpy() for k, v in st.items()}


def view(c, means, shs, opac, cov6, H, W, bg=(0, 0, 0), deg=0, colors=None):
    return orc.View(means, shs, colors, opac, cov6, c["viewmatrix"], c["projmatrix"], c["campos"],
                    float(c["tanfovx"]), float(c["tanfovy"]), np.asarray(bg, np.float32), H, W, deg)


def sh_dc(rgb):
    return ((np.asarray(rgb, np.float32) - 0.5) / 0.28209479177387814).reshape(1, 1, 3)


def test_single_isotropic_gaussian_closed_form():
    H = W = 32
    c = cam(H, W)
    z, sigma, o = 4.0, 0.05, 0.8
    means = np.array([[0, 0, z]], np.float32)
    cov6 = np.array([[sigma ** 2, 0, 0, sigma ** 2, 0, sigma ** 2]], np.float32)
    v = view(c, means, sh_dc([0.2, 0.6, 0.9]), np.array([o], np.float32), cov6, H, W, bg=(0.1, 0.1, 0.1))
    img, T, n = v.image()
    g = v.geom()
    f = W / (2 * float(c["tanfovx"]))
    s2 = (f * sigma / z) ** 2 + 0.3
    # isotropic: mid^2 - det = 0 -> disc = sqrt(0.1)
    assert g["radii"][0] == math.ceil(3 * math.sqrt(s2 + math.sqrt(0.1)))
    cx = cy = (W - 1) / 2
    assert abs(g["xy"][0, 0] - cx) < 1e-4 and abs(g["xy"][0, 1] - cy) < 1e-4
    np.testing.assert_allclose(g["conic_opacity"][0], [1 / s2, 0, 1 / s2, o], rtol=1e-5, atol=1e-7)
    ys, xs = np.mgrid[0:H, 0:W].astype(np.float64)
    alpha = np.minimum(0.99, o * np.exp(-0.5 * ((xs - cx) ** 2 + (ys - cy) ** 2) / s2))
    alpha[alpha < 1 / 255] = 0
    r = g["radii"][0]
    tiles_in = np.zeros((H, W), bool)  # tile-rect membership
    x0, x1 = max(0, int((cx - r) / 16)), min(2, int((cx + r + 15) / 16))
    tiles_in[:, x0 * 16:x1 * 16] = True
    alpha[~tiles_in] = 0
    want = alpha[None] * np.array([0.2, 0.6, 0.9])[:, None, None] + (1 - alpha[None]) * 0.1
    np.testing.assert_allclose(img, want, atol=2e-6)
    np.testing.assert_allclose(T, 1 - alpha, atol=2e-6)
    assert set(np.unique(n)) <= {0, 1}


def test_empty_scene_is_background():
    H, W = 20, 36
    c = cam(H, W)
    means = np.array([[0, 0, -3.0], [0.1, 0, 0.1]], np.float32)  # behind / in front of the 0.2 plane
    cov6 = np.tile(np.array([[0.01, 0, 0, 0.01, 0, 0.01]], np.float32), (2, 1))
    v = view(c, means, sh_dc([1, 1, 1]).repeat(2, 0), np.ones(2, np.float32) * 0.9, cov6, H, W, bg=(0.3, 0.2, 0.1))
    img, T, n = v.image()
    assert v.num_rendered == 0
    np.testing.assert_array_equal(img, np.broadcast_to(np.array([0.3, 0.2, 0.1], np.float32)[:, None, None],
                                                       img.shape))
    assert (T == 1).all() and (n == 0).all()
    assert (v.geom()["radii"] == 0).all()


def test_depth_order_not_input_order():
    H = W = 16
    c = cam(H, W)
    means = np.array([[0, 0, 5.0], [0, 0, 3.0]], np.float32)
    cov6 = np.tile(np.array([[0.02, 0, 0, 0.02, 0, 0.02]], np.float32), (2, 1))
    shs = np.concatenate([sh_dc([1, 0, 0]), sh_dc([0, 0, 1])])
    op = np.array([0.9, 0.7], np.float32)
    a = view(c, means, shs, op, cov6, H, W).image()[0]
    perm = [1, 0]
    b = view(c, means[perm], shs[perm], op[perm], cov6[perm], H, W).image()[0]
    np.testing.assert_array_equal(a, b)
    # the nearer (blue) Gaussian dominates the centre pixel
    assert a[2, 7, 7] > a[0, 7, 7]


def test_transmittance_termination():
    H = W = 15  # centre pixel (7, 7) sits exactly on the projected means
    c = cam(H, W)
    k = 5
    means = np.array([[0, 0, 2.0 + 0.1 * i] for i in range(k)], np.float32)
    cov6 = np.tile(np.array([[0.5, 0, 0, 0.5, 0, 0.5]], np.float32), (k, 1))
    v = view(c, means, sh_dc([0.5, 0.5, 0.5]).repeat(k, 0), np.full(k, 0.99, np.float32), cov6, H, W)
    _, T, n = v.image()
    # alpha = 0.99f (= 0.990000009) at the centre: T 1 -> 0.0099999905; the next Gaussian
    # would give T(1 - a) = 9.99998e-5 < 1e-4, so compositing stops after ONE contributor
    a = np.float32(0.99)
    assert n[7, 7] == 1 and T[7, 7] == np.float32(1) * (np.float32(1) - a)
    # a slightly less opaque stack needs two: T = (1 - a)^2 > 1e-4 is still blended
    v2 = view(c, means, sh_dc([0.5, 0.5, 0.5]).repeat(k, 0), np.full(k, 0.985, np.float32), cov6, H, W)
    _, T2, n2 = v2.image()
    assert n2[7, 7] == 2 and abs(T2[7, 7] - (1 - 0.985) ** 2) < 1e-7


def test_binning_sorted_and_complete():
    H, W = 48, 64
    c = cam(H, W)
    g = torch.Generator().manual_seed(3)
    P = 300
    means = (torch.randn(P, 3, generator=g) * torch.tensor([0.8, 0.6, 1.0]) + torch.tensor([0, 0, 4.0])).numpy()
    A = torch.randn(P, 3, 3, generator=g) * 0.05
    cv = (A @ A.transpose(1, 2) + 1e-4 * torch.eye(3)).numpy()
    cov6 = cv[:, [0, 0, 0, 1, 1, 2], [0, 1, 2, 1, 2, 2]].astype(np.float32)
    v = view(c, means, sh_dc([0.5, 0.5, 0.5]).repeat(P, 0), np.full(P, 0.5, np.float32), cov6, H, W)
    keys, vals, ranges = v.binning()
    gm = v.geom()
    assert v.num_rendered == int(gm["tiles_touched"][gm["radii"] > 0].sum())
    assert (np.diff(keys.astype(np.float64)) >= 0).all() and (keys[1:] >= keys[:-1]).all()
    for t, (b, e) in enumerate(ranges):
        assert ((keys[b:e] >> np.uint64(32)) == t).all()
        d = gm["depth"][vals[b:e]]
        assert (np.diff(d) >= 0).all()


def _scene(P=12, seed=0, H=24, W=32):
    g = torch.Generator().manual_seed(seed)
    means = torch.randn(P, 3, generator=g, dtype=torch.float64) * torch.tensor([0.5, 0.4, 0.5],
                                                                                dtype=torch.float64)
    means = means + torch.tensor([0, 0, 3.0], dtype=torch.float64)
    A = torch.randn(P, 3, 3, generator=g, dtype=torch.float64) * 0.08
    cov = A @ A.transpose(1, 2) + 2e-3 * torch.eye(3, dtype=torch.float64)
    cov6 = cov[:, [0, 0, 0, 1, 1, 2], [0, 1, 2, 1, 2, 2]]
    shs = torch.randn(P, 9, 3, generator=g, dtype=torch.float64) * 0.4
    opac = torch.rand(P, generator=g, dtype=torch.float64) * 0.85 + 0.05
    return means, shs, opac, cov6


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_forward_and_backward_vs_autograd(seed):
    H, W = 24, 32
    c2w = torch.eye(4)
    c2w[:3, 3] = torch.tensor([0.05, -0.03, 0.1])
    c = cam(H, W, fx=1.1, fy=1.0, c2w=c2w)
    means, shs, opac, cov6 = _scene(seed=seed, H=H, W=W)
    f32 = lambda t: t.detach().float().numpy()  # noqa: E731
    bg = np.array([0.1, 0.2, 0.3], np.float32)
    v = view(c, f32(means), f32(shs), f32(opac), f32(cov6), H, W, bg=bg, deg=2)
    img, _, _ = v.image()
    # dense reference in float64 on the SAME float32-rounded inputs
    m = torch.tensor(f32(means), dtype=torch.float64, requires_grad=True)
    s = torch.tensor(f32(shs), dtype=torch.float64, requires_grad=True)
    o = torch.tensor(f32(opac), dtype=torch.float64, requires_grad=True)
    cv = torch.tensor(f32(cov6), dtype=torch.float64, requires_grad=True)
    off = torch.zeros(m.shape[0], 2, dtype=torch.float64, requires_grad=True)
    T64 = lambda a: torch.tensor(np.asarray(a, np.float32), dtype=torch.float64)  # noqa: E731
    ref = dense_raster.render(m, s, o, cv, T64(c["viewmatrix"]).reshape(-1), T64(c["projmatrix"]).reshape(-1),
                              T64(c["campos"]), float(c["tanfovx"]), float(c["tanfovy"]), T64(bg), H, W, off)
    np.testing.assert_allclose(img, ref.detach().numpy(), atol=2e-5)
    gpix = torch.randn(3, H, W, generator=torch.Generator().manual_seed(9), dtype=torch.float64)
    (ref * gpix).sum().backward()
    gr = v.backward(gpix.float().numpy())

    def chk(got, want, name, tol=2e-3):
        want = want.detach().numpy()
        err = np.abs(got - want).max() / (np.abs(want).max() + 1e-12)
        assert err < tol, (name, err)

    chk(gr["dmean3D"], m.grad, "means")
    chk(gr["dcov6"], cv.grad, "cov6")
    chk(gr["dsh"], s.grad, "sh")
    chk(gr["dopacity"], o.grad, "opacity")
    chk(gr["dmean2D"][:, :2], off.grad, "means2D")


@pytest.mark.parametrize("shape", ["regular", "needle", "tiny"])
def test_conic_gradient_forms_agree(shape):
    """The conic-inverse gradient of the kernels and of the oracle's backward (-S G S with the
    stored conic) against upstream's computeCov2DCUDA formula through
    denom2inv = 1 / (det^2 + 1e-7) [U], both in double (oracle orc_conic_grad), and both
    against central differences of L = gA A + 2 gB B + gC C (the render backward's dconic
    convention: gB is half the derivative w.r.t. the off-diagonal entry). regular: well
    conditioned; needle: det(cov2D) ~ 4e-3 a c (the synthetic scenes' Gaussians); tiny: the
    0.3 px dilation floor, where the 1e-7 regulariser matters most (~1e-5 relative)."""
    from oracle.raster import conic_grad
    rng = np.random.default_rng({"regular": 0, "needle": 1, "tiny": 2}[shape])
    for _ in range(20):
        if shape == "regular":
            a, c = rng.uniform(0.5, 20, 2)
            b = rng.uniform(-0.5, 0.5) * np.sqrt(a * c)
        elif shape == "needle":
            a, c = rng.uniform(50, 500, 2)
            b = np.sqrt(a * c) * (1 - rng.uniform(1e-3, 5e-3)) * rng.choice([-1, 1])
        else:
            a, c = rng.uniform(0.0, 0.3, 2)
            b = rng.uniform(-0.2, 0.2) * np.sqrt(a * c)
        a, c = a + 0.3, c + 0.3
        g = rng.normal(size=3)
        f0, f1 = conic_grad(a, b, c, g, 0), conic_grad(a, b, c, g, 1)

        def L(a_, b_, c_):
            det = a_ * c_ - b_ * b_
            return g[0] * c_ / det - 2 * g[1] * b_ / det + g[2] * a_ / det
        h = 1e-6 * max(a, c)
        fd = np.array([(L(a + h, b, c) - L(a - h, b, c)) / (2 * h), (L(a, b + h, c) - L(a, b - h, c)) / (2 * h),
                       (L(a, b, c + h) - L(a, b, c - h)) / (2 * h)])
        scale = np.abs(f0).max()
        assert np.abs(f0 - f1).max() <= 2e-5 * scale, (shape, f0, f1)
        assert np.abs(f0 - fd).max() <= 1e-5 * scale, (shape, f0, fd)
