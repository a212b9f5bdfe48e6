"""Shared scene construction for the rasterizer parity tests (HIP vs oracle).

Cameras are built ONCE on the CPU with the reference's wrapper math
(my_depthsplat_amd.cuda_splatting.camera_settings) and the same float32 matrices are fed
to both the oracle and the HIP kernels, so the preprocess outputs and sort keys can be
compared bit for bit.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from my_depthsplat_amd.cuda_splatting import _cov6, camera_settings
from my_depthsplat_amd.synthetic import make_scene


def scene_inputs(h=64, w=64, n_ctx=2, n_tgt=2, seed=0, sh_degree=2, batch=1):
    sc = make_scene(batch=batch, n_context=n_ctx, n_targets=n_tgt, height=h, width=w, seed=seed, device="cpu",
                    sh_degree=sh_degree)
    return sc


def settings_for(sc, scale_invariant=True):
    B, v = sc.target_extrinsics.shape[:2]
    st = camera_settings(sc.target_extrinsics.reshape(B * v, 4, 4), sc.target_intrinsics.reshape(B * v, 3, 3),
                         sc.near.reshape(B * v), sc.far.reshape(B * v), scale_invariant)
    return {k: t.contiguous() for k, t in st.items()}


def flat_inputs(sc):
    g = sc.gaussians
    shs = g.harmonics.transpose(-1, -2).contiguous()  # [S, G, n, 3]
    return g.means.contiguous(), shs, g.opacities.contiguous(), _cov6(g.covariances).contiguous()


def oracle_views(sc, st, bg=(0.0, 0.0, 0.0), use_sh=True):
    from oracle import raster as orc
    means, shs, opac, cov6 = flat_inputs(sc)
    B, v = sc.target_extrinsics.shape[:2]
    h, w = sc.image_shape
    deg = math.isqrt(shs.shape[2]) - 1
    out = []
    npst = {k: t.numpy() for k, t in st.items()}
    for i in range(B * v):
        b = i // v
        out.append(orc.render_settings(means[b].numpy(), shs[b].numpy() if use_sh else None,
                                       None if use_sh else shs[b, :, 0, :].numpy(), opac[b].numpy(),
                                       cov6[b].numpy(), npst, i, np.asarray(bg, np.float32), h, w, deg))
    return out


def packed_cams(st, view_scene, bg=(0.0, 0.0, 0.0)):
    from my_depthsplat_amd import raster
    V = st["viewmatrix"].shape[0]
    return raster.pack_cameras(st["viewmatrix"], st["projmatrix"], st["campos"], st["tanfovx"], st["tanfovy"],
                               torch.tensor(bg, dtype=torch.float32).expand(V, 3),
                               torch.tensor(view_scene, dtype=torch.int32), st["scale"])
