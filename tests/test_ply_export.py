"""`.ply` export (drop-in for src/model/ply_export.py): header / attribute layout and the
per-attribute transforms, checked against direct numpy / scipy restatements of
ply_export.py:26-69, and the vertex arrays bit for bit against the reference's own
(tests/golden/ply.npz: make_golden.py ran ply_export.py with a recording `plyfile` stub and
real scipy). The byte layout of the file follows the PLY spec (plyfile itself is absent)."""
import numpy as np
import torch
from scipy.spatial.transform import Rotation

from my_depthsplat_amd.ply_export import (construct_list_of_attributes, export_ply, read_vertex_ply,
                                          save_gaussian_ply)


def test_attribute_list_matches_reference_order():
    assert construct_list_of_attributes(0) == ["x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2",
                                               "opacity", "scale_0", "scale_1", "scale_2",
                                               "rot_0", "rot_1", "rot_2", "rot_3"]
    assert construct_list_of_attributes(2)[9:11] == ["f_rest_0", "f_rest_1"]


def test_export_ply_values(tmp_path):
    g = torch.Generator().manual_seed(0)
    G = 50
    ext = torch.eye(4)
    ext[:3, :3] = torch.from_numpy(Rotation.from_euler("xyz", [0.3, -0.2, 0.5]).as_matrix()).float()
    ext[:3, 3] = torch.tensor([0.1, 0.2, 0.3])
    means = torch.randn(G, 3, generator=g)
    scales = torch.rand(G, 3, generator=g) * 0.1 + 1e-3
    q = torch.randn(G, 4, generator=g)
    rot = q / q.norm(dim=-1, keepdim=True)
    harm = torch.randn(G, 3, 9, generator=g)
    opac = torch.rand(G, generator=g) * 0.98 + 0.01
    path = tmp_path / "sub" / "g.ply"
    export_ply(ext, means, scales, rot, harm, opac, path)
    raw = path.read_bytes()
    assert raw.startswith(b"ply\nformat binary_little_endian 1.0\nelement vertex 50\nproperty float x\n")
    names, vals = read_vertex_ply(path)
    assert names == construct_list_of_attributes(0) and vals.shape == (G, 17)
    Rinv = np.linalg.inv(ext[:3, :3].numpy().astype(np.float64))
    np.testing.assert_allclose(vals[:, 0:3], means.numpy() @ Rinv.T, rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(vals[:, 3:6], 0)
    np.testing.assert_allclose(vals[:, 6:9], harm[..., 0].numpy(), rtol=0, atol=0)
    np.testing.assert_allclose(vals[:, 9], np.log(opac.numpy() / (1 - opac.numpy())), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(vals[:, 10:13], np.log(scales.numpy()), rtol=1e-6, atol=1e-6)
    want = Rotation.from_matrix(Rinv @ Rotation.from_quat(rot.numpy()).as_matrix()).as_quat()  # xyzw
    got = vals[:, 13:17]  # wxyz
    np.testing.assert_allclose(np.abs((got[:, [1, 2, 3, 0]] * want).sum(-1)), 1.0, atol=1e-5)


def test_save_gaussian_ply_trims_borders(tmp_path):
    from my_depthsplat_amd.decoder import Gaussians
    v, h, w = 2, 20, 24
    G = v * h * w
    g = torch.Generator().manual_seed(1)
    gs = Gaussians(torch.randn(1, G, 3, generator=g), torch.eye(3).expand(1, G, 3, 3).clone(),
                   torch.randn(1, G, 3, 4, generator=g), torch.rand(1, G, generator=g) * 0.9 + 0.05)
    dump = {"scales": torch.rand(1, G, 3, generator=g) + 0.01, "rotations": torch.randn(1, G, 4, generator=g)}
    ext = torch.eye(4).expand(1, v, 4, 4).clone()
    example = {"context": {"image": torch.zeros(1, v, 3, h, w), "extrinsics": ext}}
    save_gaussian_ply(gs, dump, example, tmp_path / "s.ply")
    names, vals = read_vertex_ply(tmp_path / "s.ply")
    assert vals.shape[0] == v * (h - 16) * (w - 16)
    # identity cameras: positions pass through; first kept Gaussian = pixel (8, 8) of view 0
    first = gs.means[0].reshape(v, h, w, 3)[0, 8, 8].numpy()
    np.testing.assert_allclose(vals[0, 0:3], first, rtol=1e-6)


def _golden():
    from pathlib import Path
    return np.load(Path(__file__).parent / "golden" / "ply.npz")


def test_export_ply_matches_reference_fixture(tmp_path):
    """tests/golden/ply.npz: the vertex array the REFERENCE's export_ply built
    (src/model/ply_export.py:26-63, run by make_golden.py with a recording plyfile stub and
    real scipy) for a non-identity c2w; reproduced bit for bit."""
    G = _golden()
    T = lambda k: torch.from_numpy(G[k])  # noqa: E731
    path = tmp_path / "a.ply"
    export_ply(T("export_ext"), T("export_means"), T("export_scales"), T("export_rot"), T("export_harm"),
               T("export_opac"), path)
    names, vals = read_vertex_ply(path)
    assert names == construct_list_of_attributes(0)
    np.testing.assert_array_equal(vals, G["export_vertex"])


def test_save_gaussian_ply_matches_reference_fixture(tmp_path):
    """save_gaussian_ply (ply_export.py:66-115) on a 2-view 20x20 context: the 8-pixel border
    trim in the reference's "h w spp v" order (4 x 4 x 1 x 2 = 32 Gaussians), camera -> world
    rotations, first-camera frame; equal to the reference-recorded vertex array bit for bit."""
    import types
    G = _golden()
    T = lambda k: torch.from_numpy(G[k])  # noqa: E731
    v, h, w = (int(x) for x in G["save_hw"])
    gs = types.SimpleNamespace(means=T("save_means"), harmonics=T("save_harm"), opacities=T("save_opac"))
    dump = {"rotations": T("save_rot"), "scales": T("save_scales")}
    example = {"context": {"extrinsics": T("save_ext")[None], "image": torch.zeros(1, v, 3, h, w)}}
    path = tmp_path / "b.ply"
    save_gaussian_ply(gs, dump, example, path)
    names, vals = read_vertex_ply(path)
    assert vals.shape == G["save_vertex"].shape == (32, 17)
    np.testing.assert_array_equal(vals, G["save_vertex"])
