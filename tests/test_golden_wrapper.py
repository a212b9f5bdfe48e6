"""The reference wrapper semantics, pinned by fixtures recorded from the reference itself
(tests/golden/make_golden.py runs src/model/decoder/cuda_splatting.py with a recording
rasterizer stub). CPU only: this is the host-side camera / input preparation."""
from __future__ import annotations

import math
from pathlib import Path

import numpy as np
import pytest
import torch

from my_depthsplat_amd.cuda_splatting import (_cov6, camera_settings, depth_colors, get_projection_matrix,
                                              orthographic_settings)

G = np.load(Path(__file__).parent / "golden" / "cuda_splatting_settings.npz")
T = lambda k: torch.from_numpy(G[k])  # noqa: E731
B = G["extrinsics"].shape[0]


def close(a, b, rtol=1e-6, atol=1e-6):
    np.testing.assert_allclose(np.asarray(a, np.float64), np.asarray(b, np.float64), rtol=rtol, atol=atol)


def test_projection_matrix():
    near, far = T("near"), T("far")
    got = get_projection_matrix(near, far, torch.tensor([0.9, 1.2, 0.5]), torch.tensor([0.8, 1.0, 0.7]))
    close(got, G["projection_matrix"], 0, 0)


@pytest.mark.parametrize("tag,scale_invariant", [("si", True), ("ns", False)])
def test_camera_settings(tag, scale_invariant):
    st = camera_settings(T("extrinsics"), T("intrinsics"), T("near"), T("far"), scale_invariant)
    for i in range(B):
        close(st["viewmatrix"][i], G[f"{tag}_view{i}_viewmatrix"])
        close(st["projmatrix"][i], G[f"{tag}_view{i}_projmatrix"])
        close(st["campos"][i], G[f"{tag}_view{i}_campos"])
    for i in range(B):
        if tag == "si":
            close([st["tanfovx"][i], st["tanfovy"][i]], G[f"si_view{i}_tanfov"])


def test_rasterizer_inputs_scale_invariant():
    """means*scale, cov*scale^2 -> triu gather, SH 'b g xyz n -> b g n xyz', opacity[..., None]."""
    st = camera_settings(T("extrinsics"), T("intrinsics"), T("near"), T("far"), True)
    means, cov, sh, opac = T("means"), T("cov"), T("sh"), T("opacities")
    for i in range(B):
        s = st["scale"][i]
        close(means[i] * s, G[f"si_view{i}_means3D"], 0, 0)
        close(_cov6(cov[i] * s ** 2), G[f"si_view{i}_cov3D_precomp"], 0, 0)
        close(sh[i].transpose(-1, -2), G[f"si_view{i}_shs"], 0, 0)
        close(opac[i][:, None], G[f"si_view{i}_opacities"], 0, 0)
        assert int(G[f"si_view{i}_shdeg"]) == math.isqrt(sh.shape[-1]) - 1


def test_rasterizer_inputs_colors_precomp():
    sh = T("sh")[..., :1]
    for i in range(B):
        close(sh[i].transpose(-1, -2)[:, 0, :], G[f"ns_view{i}_colors_precomp"], 0, 0)
        close(_cov6(T("cov")[i]), G[f"ns_view{i}_cov3D_precomp"], 0, 0)


@pytest.mark.parametrize("mode", ["depth", "disparity", "log"])
def test_depth_colors(mode):
    """render_depth_cuda colours (in the reference they are computed BEFORE render_cuda's
    scale-invariant rescale, which only touches means/cov)."""
    c = depth_colors(T("extrinsics"), T("means"), T("near"), T("far"), mode)
    for i in range(B):
        close(c[i][:, None].expand(-1, 3), G[f"depth_{mode}_view{i}_colors_precomp"], 1e-5, 1e-6)


def test_orthographic_settings():
    st = orthographic_settings(T("extrinsics")[:1], T("ortho_width"), T("ortho_height"), T("near")[:1],
                               T("far")[:1], fov_degrees=10.0)
    close(st["viewmatrix"][0], G["ortho_view0_viewmatrix"], 1e-5, 1e-5)
    close(st["projmatrix"][0], G["ortho_view0_projmatrix"], 1e-5, 1e-5)
    close(st["campos"][0], G["ortho_view0_campos"], 1e-5, 1e-5)
    close([float(st["tanfovx"][0]), float(st["tanfovy"][0])], G["ortho_view0_tanfov"], 1e-6, 1e-7)
