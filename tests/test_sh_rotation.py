"""rotate_sh without e3nn: parity with e3nn 0.5.1 is unpinned for non-identity rotations
(e3nn absent), so the Wigner-D construction is checked by its defining
properties: D(I) = I, orthogonality, homomorphism, D_1 = R, equivariance of the basis."""
from __future__ import annotations

import math

import torch

from my_depthsplat_amd.sh_rotation import e3nn_real_sh, rotate_sh, wigner_d


def rand_rot(n, seed):
    g = torch.Generator().manual_seed(seed)
    q, _ = torch.linalg.qr(torch.randn(n, 3, 3, generator=g, dtype=torch.float64))
    q = q * torch.sign(torch.det(q))[:, None, None]
    return q


def test_identity_and_l1():
    I = torch.eye(3, dtype=torch.float64)[None]
    for l in range(4):
        assert torch.allclose(wigner_d(l, I)[0], torch.eye(2 * l + 1, dtype=torch.float64), atol=1e-12)
    R = rand_rot(5, 0)
    assert torch.allclose(wigner_d(1, R), R, atol=1e-12)


def test_orthogonal_and_homomorphism():
    R1, R2 = rand_rot(4, 1), rand_rot(4, 2)
    for l in range(4):
        D1, D2, D12 = wigner_d(l, R1), wigner_d(l, R2), wigner_d(l, R1 @ R2)
        eye = torch.eye(2 * l + 1, dtype=torch.float64).expand_as(D1)
        assert torch.allclose(D1 @ D1.transpose(-1, -2), eye, atol=1e-10)
        assert torch.allclose(D12, D1 @ D2, atol=1e-10)


def test_equivariance_of_basis():
    R = rand_rot(3, 3)
    x = torch.nn.functional.normalize(torch.randn(7, 3, dtype=torch.float64), dim=-1)
    for l in range(4):
        D = wigner_d(l, R)  # [3, m, m]
        lhs = e3nn_real_sh(l, torch.einsum("rij,nj->rni", R, x))
        rhs = torch.einsum("rkm,nm->rnk", D, e3nn_real_sh(l, x))
        assert torch.allclose(lhs, rhs, atol=1e-10)


def test_rotate_sh_shapes_and_identity():
    sh = torch.randn(2, 5, 3, 9)
    I = torch.eye(3).expand(2, 5, 1, 3, 3)
    assert torch.allclose(rotate_sh(sh, I), sh, atol=1e-6)
    R = rand_rot(1, 4).float().expand(2, 5, 1, 3, 3)
    out = rotate_sh(sh, R)
    assert out.shape == sh.shape
    # the l = 0 (DC) coefficient is rotation invariant; norms per degree are preserved
    assert torch.allclose(out[..., 0], sh[..., 0], atol=1e-6)
    for l in range(3):
        sl = slice(l * l, (l + 1) ** 2)
        assert torch.allclose(out[..., sl].norm(dim=-1), sh[..., sl].norm(dim=-1), atol=1e-5)
    assert math.isfinite(float(out.sum()))
