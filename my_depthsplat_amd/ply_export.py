"""3DGS `.ply` export: drop-in for src/model/ply_export.py.

Same functions, arguments and file layout as the reference (`construct_list_of_attributes`,
`export_ply`, `save_gaussian_ply`): one binary little-endian `vertex` element with float32
properties x y z nx ny nz f_dc_0..2 opacity scale_0..2 rot_0..3 (DC band only, normals 0,
opacity as a logit, log scales, wxyz quaternions), positions and rotations expressed in the
first context camera's rotation frame (ply_export.py:26-69). The reference writes through
`plyfile`; this writes the identical header / record stream with numpy (plyfile is not a
dependency here). Host-side I/O: the Gaussians are copied off the device once.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np
import torch
from scipy.spatial.transform import Rotation


def construct_list_of_attributes(num_rest: int) -> list[str]:
    """ply_export.py:12-23."""
    attributes = ["x", "y", "z", "nx", "ny", "nz"]
    attributes += [f"f_dc_{i}" for i in range(3)]
    attributes += [f"f_rest_{i}" for i in range(num_rest)]
    attributes.append("opacity")
    attributes += [f"scale_{i}" for i in range(3)]
    attributes += [f"rot_{i}" for i in range(4)]
    return attributes


def write_vertex_ply(path: Path, names: list[str], values: np.ndarray) -> None:
    """Binary little-endian PLY with one `vertex` element of float32 properties."""
    values = np.ascontiguousarray(values, dtype="<f4")
    header = ["ply", "format binary_little_endian 1.0", f"element vertex {values.shape[0]}"]
    header += [f"property float {n}" for n in names]
    header.append("end_header")
    path.parent.mkdir(exist_ok=True, parents=True)
    with open(path, "wb") as f:
        f.write(("\n".join(header) + "\n").encode("ascii"))
        f.write(values.tobytes())


def read_vertex_ply(path: Path) -> tuple[list[str], np.ndarray]:
    """Reader for the files write_vertex_ply produces (tests, round trips)."""
    data = Path(path).read_bytes()
    end = data.index(b"end_header\n") + len(b"end_header\n")
    lines = data[:end].decode("ascii").splitlines()
    n = int(next(l for l in lines if l.startswith("element vertex")).split()[-1])
    names = [l.split()[-1] for l in lines if l.startswith("property")]
    vals = np.frombuffer(data[end:], dtype="<f4").reshape(n, len(names))
    return names, vals


def export_ply(extrinsics: torch.Tensor, means: torch.Tensor, scales: torch.Tensor, rotations: torch.Tensor,
               harmonics: torch.Tensor, opacities: torch.Tensor, path: Path) -> None:
    """ply_export.py:26-69. extrinsics [4,4] c2w; means [G,3]; scales [G,3]; rotations [G,4]
    xyzw; harmonics [G,3,d_sh]; opacities [G]."""
    view_rotation = extrinsics[:3, :3].detach().cpu().float().inverse()
    m = torch.einsum("ij,...j->...i", view_rotation, means.detach().cpu().float()).numpy()
    rot = Rotation.from_quat(rotations.detach().cpu().numpy()).as_matrix()
    rot = view_rotation.numpy() @ rot
    x, y, z, w = Rotation.from_matrix(rot).as_quat().T
    quat = np.stack((w, x, y, z), axis=-1)
    dc = harmonics[..., 0].detach().cpu().numpy()
    attrs = np.concatenate([m, np.zeros_like(m), dc, torch.logit(opacities[..., None].detach()).cpu().numpy(),
                            scales.detach().log().cpu().numpy(), quat], axis=1)
    write_vertex_ply(Path(path), construct_list_of_attributes(0), attrs)


def save_gaussian_ply(gaussians, visualization_dump: dict, example: dict, save_path: Path) -> None:
    """ply_export.py:72-115: trim 8 border pixels of every context view, bring the
    camera-space rotations to world space, export in the first context camera's frame."""
    v, _, h, w = example["context"]["image"].shape[1:]
    trim_px = 8
    mask = torch.zeros((h, w, 1, v), dtype=torch.bool)
    mask[trim_px:-trim_px, trim_px:-trim_px] = True

    def trim(t):  # "() (v h w spp) ... -> h w spp v ..." then mask
        t = t.detach().cpu()
        rest = t.shape[1:]
        t = t.reshape(v, h, w, 1, *rest).permute(1, 2, 3, 0, *range(4, 4 + len(rest)))
        return t[mask]

    cam_rot = trim(visualization_dump["rotations"][0])
    c2w = example["context"]["extrinsics"][0, :, :3, :3].detach().cpu()
    c2w = c2w[None, None, None].expand(h, w, 1, v, 3, 3)[mask]
    world = c2w.double().numpy() @ Rotation.from_quat(cam_rot.numpy()).as_matrix()
    world_q = torch.from_numpy(Rotation.from_matrix(world).as_quat()).float()
    export_ply(example["context"]["extrinsics"][0, 0], trim(gaussians.means[0]), trim(visualization_dump["scales"][0]),
               world_q, trim(gaussians.harmonics[0]), trim(gaussians.opacities[0]), save_path)
