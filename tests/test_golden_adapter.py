"""Gaussian adapter + camera helpers vs fixtures produced by the reference itself
(tests/golden/make_golden.py; identity c2w rotations because e3nn is absent)."""
from __future__ import annotations

from pathlib import Path

import numpy as np
import torch

from my_depthsplat_amd.gaussian_adapter import (GaussianAdapter, GaussianAdapterCfg, build_covariance,
                                                quaternion_to_matrix)
from my_depthsplat_amd.projection import get_fov, get_world_rays, sample_image_grid

G = np.load(Path(__file__).parent / "golden" / "adapter.npz")
T = lambda k: torch.from_numpy(G[k])  # noqa: E731


def close(a, b, rtol=1e-6, atol=1e-6):
    np.testing.assert_allclose(np.asarray(a), np.asarray(b), rtol=rtol, atol=atol)


def test_adapter_forward():
    ad = GaussianAdapter(GaussianAdapterCfg(1e-10, 3.0, 2))
    e = T("extrinsics")[:, :, None, None, None]
    k = T("intrinsics")[:, :, None, None, None]
    h, w = G["images"].shape[-2:]
    out = ad(e, k, T("coordinates"), T("depths"), T("opacities"), T("raw"), (h, w), input_images=T("images"))
    close(out.means, G["means"], 1e-5, 1e-5)
    close(out.covariances, G["covariances"], 1e-5, 1e-7)
    close(out.harmonics, G["harmonics"], 1e-5, 1e-6)
    close(out.scales, G["scales"])
    close(out.rotations, G["rotations"])
    close(out.opacities, G["out_opacities"], 0, 0)


def test_quaternion_and_covariance():
    close(quaternion_to_matrix(T("quat")), G["quat_matrix"])
    close(build_covariance(T("scale3"), T("quat")), G["build_cov"], 1e-5, 1e-7)


def test_rays_fov_grid():
    e = T("extrinsics")[:, :, None, None, None]
    k = T("intrinsics")[:, :, None, None, None]
    o, d = get_world_rays(T("coordinates"), e, k)
    close(o, G["rays_o"])
    close(d, G["rays_d"], 1e-6, 1e-6)
    close(get_fov(T("fov_K")), G["fov"])
    h, w = G["images"].shape[-2:]
    xy, ij = sample_image_grid((h, w))
    close(xy, G["grid_xy"], 0, 0)
    assert np.array_equal(ij.numpy(), G["grid_ij"])
