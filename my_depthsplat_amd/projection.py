"""Camera helpers used around the hot path (host-side torch, not kernels).

Restates the subset of src/geometry/projection.py the decoder and the Gaussian adapter
depend on (SURVEY.md §2 row "src/geometry/ (partial)"):
  homogenize_points / homogenize_vectors  projection.py:9-20
  unproject                               projection.py:74-88
  get_world_rays                          projection.py:91-114
  sample_image_grid                       projection.py:117-137
  get_fov                                 projection.py:233-247
Semantics (shapes, broadcasting, normalisation order) follow the reference so the
golden fixtures in tests/golden/ pin them.
"""
from __future__ import annotations

import torch


def homogenize_points(points: torch.Tensor) -> torch.Tensor:
    """xyz -> xyz1 (projection.py:9-13)."""
    return torch.cat([points, points.new_ones(points.shape[:-1] + (1,))], dim=-1)


def homogenize_vectors(vectors: torch.Tensor) -> torch.Tensor:
    """xyz -> xyz0 (projection.py:16-20)."""
    return torch.cat([vectors, vectors.new_zeros(vectors.shape[:-1] + (1,))], dim=-1)


def _apply(mat: torch.Tensor, vec: torch.Tensor) -> torch.Tensor:
    # "... i j, ... j -> ... i" with broadcasting of the batch dims
    return torch.einsum("...ij,...j->...i", mat, vec)


def unproject(coordinates: torch.Tensor, z: torch.Tensor, intrinsics: torch.Tensor) -> torch.Tensor:
    """Camera-space points at depth z through K^-1 (projection.py:74-88)."""
    rays = _apply(intrinsics.inverse(), homogenize_points(coordinates))
    return rays * z[..., None]


def get_world_rays(coordinates: torch.Tensor, extrinsics: torch.Tensor,
                   intrinsics: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """(origins, directions) in world space; directions scaled so camera-space z = 1
    (projection.py:91-114)."""
    d = unproject(coordinates, torch.ones_like(coordinates[..., 0]), intrinsics)
    d = d / d[..., -1:]
    d = _apply(extrinsics, homogenize_vectors(d))[..., :-1]
    origins = extrinsics[..., :-1, -1].broadcast_to(d.shape)
    return origins, d


def sample_image_grid(shape: tuple[int, ...], device: torch.device = torch.device("cpu")):
    """Pixel-centre coordinates in (0, 1), xy order, plus integer ij indices
    (projection.py:117-137)."""
    idx = [torch.arange(n, device=device) for n in shape]
    ij = torch.stack(torch.meshgrid(*idx, indexing="ij"), dim=-1)
    centres = [(i + 0.5) / n for i, n in zip(idx, shape)]
    xy = torch.stack(torch.meshgrid(*reversed(centres), indexing="xy"), dim=-1)
    return xy, ij


def get_fov(intrinsics: torch.Tensor) -> torch.Tensor:
    """[b, 3, 3] normalised intrinsics -> [b, 2] (fov_x, fov_y) from the image-edge
    midpoints (projection.py:233-247). Assumes a centred principal point, as the
    rasterizer only takes tan(fov/2)."""
    kinv = intrinsics.inverse()

    def ray(v):
        r = torch.einsum("bij,j->bi", kinv, torch.tensor(v, dtype=torch.float32, device=intrinsics.device))
        return r / r.norm(dim=-1, keepdim=True)

    fx = (ray([0, 0.5, 1]) * ray([1, 0.5, 1])).sum(dim=-1).acos()
    fy = (ray([0.5, 0, 1]) * ray([0.5, 1, 1])).sum(dim=-1).acos()
    return torch.stack((fx, fy), dim=-1)
