"""rotate_sh without e3nn (drop-in for src/misc/sh_rotation.py:10-30).

The reference rotates SH coefficients with e3nn 0.5.1 (`matrix_to_angles` + `wigner_D`,
requirements.txt:5), which is not installed here. A Wigner-D matrix is fully determined
by the real-SH basis it acts on: D_l(R) is the unique matrix with
Y_l(R x) = D_l(R) Y_l(x) for all unit x. We build it from e3nn's own real spherical
harmonics (y-polar convention; l = 1 components ordered (x, y, z), so D_1(R) = R) by
solving that identity on a fixed, well-conditioned set of directions.

PARITY: unpinned for non-identity rotations (no e3nn output exists on disk). Checked by
properties instead: D(I) = I, orthogonality, D(R1 R2) = D(R1) D(R2), D_1 = R, and the
defining equivariance identity (tests/test_sh_rotation.py). Identity rotations are
pinned by tests/golden/adapter.npz.
"""
from __future__ import annotations

import math
from functools import lru_cache

import torch


def e3nn_real_sh(l: int, xyz: torch.Tensor) -> torch.Tensor:
    """e3nn-convention real spherical harmonics of degree l (unnormalised per degree,
    which does not change D). xyz [..., 3] -> [..., 2l+1]."""
    x, y, z = xyz.unbind(-1)
    if l == 0:
        return torch.ones_like(x)[..., None]
    if l == 1:
        return torch.stack([x, y, z], dim=-1)
    s3 = math.sqrt(3.0)
    y2 = y * y
    x2z2 = x * x + z * z
    s20 = s3 * x * z
    s24 = s3 / 2.0 * (z * z - x * x)
    if l == 2:
        return torch.stack([s20, s3 * x * y, y2 - 0.5 * x2z2, s3 * y * z, s24], dim=-1)
    if l == 3:
        return torch.stack([
            math.sqrt(5 / 6) * (s20 * z + s24 * x),
            math.sqrt(5) * s20 * y,
            math.sqrt(3 / 8) * (4 * y2 - x2z2) * x,
            0.5 * y * (2 * y2 - 3 * x2z2),
            math.sqrt(3 / 8) * z * (4 * y2 - x2z2),
            math.sqrt(5) * s24 * y,
            math.sqrt(5 / 6) * (s24 * z - s20 * x),
        ], dim=-1)
    raise ValueError(f"rotate_sh supports degrees 0..3, got {l}")


@lru_cache(maxsize=None)
def _probe(l: int):
    g = torch.Generator().manual_seed(1234 + l)
    pts = torch.randn(4 * (2 * l + 1) + 8, 3, generator=g, dtype=torch.float64)
    pts = pts / pts.norm(dim=-1, keepdim=True)
    Y = e3nn_real_sh(l, pts)                 # [N, 2l+1]
    return pts, torch.linalg.pinv(Y)         # pinv: [2l+1, N]


def wigner_d(l: int, rotations: torch.Tensor) -> torch.Tensor:
    """D_l(R) for rotations [..., 3, 3] -> [..., 2l+1, 2l+1] (float64 internally)."""
    if l == 0:
        return torch.ones(rotations.shape[:-2] + (1, 1), dtype=rotations.dtype, device=rotations.device)
    pts, pinv = _probe(l)
    R = rotations.to(torch.float64)
    pts = pts.to(R.device)
    rotated = torch.einsum("...ij,nj->...ni", R, pts)          # R x_n
    Yr = e3nn_real_sh(l, rotated)                              # [..., N, 2l+1]
    D = torch.einsum("...nk,mn->...km", Yr, pinv.to(R.device))  # Y(Rx)^T pinv(Y(x))^T
    return D.to(rotations.dtype)


def rotate_sh(sh_coefficients: torch.Tensor, rotations: torch.Tensor) -> torch.Tensor:
    """sh [..., n] (n = (deg+1)^2), rotations [..., 3, 3] (broadcastable) -> [..., n]."""
    n = sh_coefficients.shape[-1]
    out = []
    for l in range(math.isqrt(n)):
        D = wigner_d(l, rotations).to(sh_coefficients.dtype)
        out.append(torch.einsum("...ij,...j->...i", D, sh_coefficients[..., l * l:(l + 1) ** 2]))
    return torch.cat(out, dim=-1)
