#!/usr/bin/env python
"""Generate the golden fixtures in tests/golden/ by RUNNING THE REFERENCE in this container.

Run from the repo root in the build container (where /root/reference exists):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
The reference never travels: only the resulting .npz data files are committed.

Missing third-party modules are replaced by tiny stubs written to a temp dir:
  jaxtyping                 annotations only (no runtime checking)
  torchvision.transforms    placeholder (imported but unused by the pieces run here)
  e3nn.o3                   identity-only: matrix_to_angles asserts R == I, wigner_D = I
                            (so adapter fixtures use identity c2w rotations)
  diff_gaussian_rasterization   RECORDING stub: stores every GaussianRasterizationSettings
                            and the tensors handed to the rasterizer, returns zeros. This
                            pins the reference wrapper (cuda_splatting.py:46-264) exactly.
  plyfile                   RECORDING stub: PlyElement.describe keeps the structured vertex
                            array the reference builds, PlyData.write records it (no file
                            format is written; the values pin ply_export.py:26-115).
Reference packages are mounted as namespace packages (their __init__ chains import
lightning / datasets and are skipped), following SURVEY.md Appendix A.
"""
from __future__ import annotations

import importlib
import os
import sys
import tempfile
import types
from pathlib import Path

import numpy as np
import torch

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent

STUBS = {
    "jaxtyping/__init__.py": """
class _A:
    def __class_getitem__(cls, item):
        return object
Float = Int64 = Bool = Shaped = UInt8 = Int = Float32 = Integer = _A
import contextlib
@contextlib.contextmanager
def install_import_hook(*a, **k):
    yield
""",
    "torchvision/__init__.py": "",
    "torchvision/transforms.py": "class Pad:\n    def __init__(self, *a, **k):\n        pass\n",
    "e3nn/__init__.py": "",
    "e3nn/o3.py": """
import torch
def matrix_to_angles(R):
    eye = torch.eye(3, dtype=R.dtype, device=R.device).expand_as(R)
    assert torch.allclose(R, eye), "identity-only e3nn stub"
    z = torch.zeros(R.shape[:-2], dtype=R.dtype, device=R.device)
    return z, z, z
def wigner_D(l, a, b, c):
    return torch.eye(2 * l + 1, dtype=a.dtype, device=a.device).expand(*a.shape, 2 * l + 1, 2 * l + 1)
""",
    "diff_gaussian_rasterization/__init__.py": """
import torch
from typing import NamedTuple
RECORD = []
class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool
class GaussianRasterizer(torch.nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings
    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None):
        RECORD.append(dict(settings=self.raster_settings, means3D=means3D.detach().clone(),
                           shs=None if shs is None else shs.detach().clone(),
                           colors_precomp=None if colors_precomp is None else colors_precomp.detach().clone(),
                           opacities=opacities.detach().clone(), cov3D_precomp=cov3D_precomp.detach().clone()))
        s = self.raster_settings
        img = torch.zeros(3, s.image_height, s.image_width) + 0 * means3D.sum()
        return img, torch.zeros(means3D.shape[0], dtype=torch.int32)
""",
    "plyfile/__init__.py": """
RECORD = []
class PlyElement:
    def __init__(self, data, name):
        self.data, self.name = data, name
    @staticmethod
    def describe(data, name, **kw):
        return PlyElement(data.copy(), name)
class PlyData:
    def __init__(self, elements, **kw):
        self.elements = list(elements)
    def write(self, path):
        RECORD.append((str(path), [(e.name, e.data) for e in self.elements]))
""",
}


def setup_imports():
    tmp = Path(tempfile.mkdtemp(prefix="dsplat_stubs_"))
    for rel, txt in STUBS.items():
        p = tmp / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(txt)
    sys.path.insert(0, str(tmp))
    sys.dont_write_bytecode = True
    for pkg in ["src", "src.model", "src.model.decoder", "src.model.encoder", "src.model.encoder.common",
                "src.model.encoder.unimatch", "src.geometry", "src.misc", "src.dataset"]:
        m = types.ModuleType(pkg)
        m.__path__ = [str(REF / pkg.replace(".", "/"))]
        sys.modules[pkg] = m
    # decoder_splatting_cuda imports `from ...dataset import DatasetCfg` (a type only)
    sys.modules["src.dataset"].DatasetCfg = object


def t2n(x):
    return x.detach().cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x)


def gen_cuda_splatting():
    cs = importlib.import_module("src.model.decoder.cuda_splatting")
    rec = importlib.import_module("diff_gaussian_rasterization").RECORD
    g = torch.Generator().manual_seed(0)
    b, G, n = 3, 40, 9
    ext = torch.eye(4).repeat(b, 1, 1)
    ang = torch.rand(b, generator=g) * 0.6 - 0.3
    ext[:, 0, 0], ext[:, 0, 2], ext[:, 2, 0], ext[:, 2, 2] = ang.cos(), ang.sin(), -ang.sin(), ang.cos()
    ext[:, :3, 3] = torch.randn(b, 3, generator=g) * 0.3
    K = torch.tensor([[1.0, 0, 0.5], [0, 1.1, 0.5], [0, 0, 1]]).repeat(b, 1, 1)
    near = torch.tensor([0.5, 1.0, 0.25])
    far = torch.tensor([100.0, 50.0, 10.0])
    bg = torch.rand(b, 3, generator=g)
    means = torch.randn(b, G, 3, generator=g) + torch.tensor([0, 0, 4.0])
    A = torch.randn(b, G, 3, 3, generator=g) * 0.1
    cov = A @ A.transpose(-1, -2) + 1e-3 * torch.eye(3)
    sh = torch.randn(b, G, 3, n, generator=g)
    opac = torch.rand(b, G, generator=g)
    out = {"extrinsics": ext, "intrinsics": K, "near": near, "far": far, "bg": bg, "means": means, "cov": cov,
           "sh": sh, "opacities": opac, "image_hw": np.array([24, 40])}
    rec.clear()
    cs.render_cuda(ext, K, near, far, (24, 40), bg, means, cov, sh, opac, scale_invariant=True, use_sh=True)
    for i, r in enumerate(rec):
        s = r["settings"]
        out[f"si_view{i}_viewmatrix"] = s.viewmatrix
        out[f"si_view{i}_projmatrix"] = s.projmatrix
        out[f"si_view{i}_campos"] = s.campos
        out[f"si_view{i}_tanfov"] = np.array([s.tanfovx, s.tanfovy], np.float64)
        out[f"si_view{i}_shdeg"] = np.array(s.sh_degree)
        out[f"si_view{i}_bg"] = s.bg
        for k in ("means3D", "shs", "opacities", "cov3D_precomp"):
            out[f"si_view{i}_{k}"] = r[k]
    rec.clear()
    cs.render_cuda(ext, K, near, far, (24, 40), bg, means, cov, sh[..., :1], opac, scale_invariant=False,
                   use_sh=False)
    for i, r in enumerate(rec):
        s = r["settings"]
        out[f"ns_view{i}_viewmatrix"] = s.viewmatrix
        out[f"ns_view{i}_projmatrix"] = s.projmatrix
        out[f"ns_view{i}_campos"] = s.campos
        out[f"ns_view{i}_colors_precomp"] = r["colors_precomp"]
        out[f"ns_view{i}_means3D"] = r["means3D"]
        out[f"ns_view{i}_cov3D_precomp"] = r["cov3D_precomp"]
    for mode in ("depth", "disparity", "log"):
        rec.clear()
        cs.render_depth_cuda(ext, K, near, far, (24, 40), means, cov, opac, mode=mode)
        for i, r in enumerate(rec):
            out[f"depth_{mode}_view{i}_colors_precomp"] = r["colors_precomp"]
            out[f"depth_{mode}_view{i}_means3D"] = r["means3D"]
    rec.clear()
    # the reference's orthographic path only supports b = 1 (move_back[2, 3] = -distance)
    width = torch.tensor([2.0])
    height = torch.tensor([1.0])
    cs.render_cuda_orthographic(ext[:1], width, height, near[:1], far[:1], (24, 40), bg[:1], means[:1], cov[:1],
                                sh[:1], opac[:1], fov_degrees=10.0)
    out["ortho_width"], out["ortho_height"] = width, height
    for i, r in enumerate(rec):
        s = r["settings"]
        out[f"ortho_view{i}_viewmatrix"] = s.viewmatrix
        out[f"ortho_view{i}_projmatrix"] = s.projmatrix
        out[f"ortho_view{i}_campos"] = s.campos
        out[f"ortho_view{i}_tanfov"] = np.array([float(s.tanfovx), float(s.tanfovy)], np.float64)
    out["projection_matrix"] = cs.get_projection_matrix(near, far, torch.tensor([0.9, 1.2, 0.5]),
                                                        torch.tensor([0.8, 1.0, 0.7]))
    np.savez_compressed(OUT / "cuda_splatting_settings.npz", **{k: t2n(v) for k, v in out.items()})


def gen_cost_volume():
    mt = importlib.import_module("src.model.encoder.unimatch.matching")
    mvt = importlib.import_module("src.model.encoder.unimatch.mv_transformer")
    g = torch.Generator().manual_seed(1)
    out = {}
    for tag, (B, V, C, H, W, D, per_pixel) in {"s0": (1, 3, 16, 12, 16, 8, False),
                                               "s1": (2, 2, 8, 10, 14, 4, True)}.items():
        feats = [torch.randn(B, C, H, W, generator=g) for _ in range(V)]
        K = torch.tensor([[W * 0.9, 0, W / 2], [0, H * 0.9, H / 2], [0, 0, 1.0]])
        intr = [K.expand(B, 3, 3).clone() for _ in range(V)]
        extr = []
        for v in range(V):
            e = torch.eye(4).expand(B, 4, 4).clone()
            e[:, 0, 3] = 0.1 * v
            e[:, 1, 3] = 0.03 * v
            extr.append(e)
        ref, ref_k, ref_e, tgt, tgt_k, tgt_e = mvt.batch_features_camera_parameters(feats, intr, extr)
        BV, J = tgt.shape[:2]
        pose = torch.matmul(tgt_e.inverse(), ref_e.unsqueeze(1))
        inv_min, inv_max = 1 / 10.0, 1 / 0.5
        if per_pixel:
            inv = inv_min + torch.rand(BV, D, H, W, generator=g) * (inv_max - inv_min)
        else:
            inv = (inv_min + torch.linspace(0, 1, D).view(1, D, 1, 1) * (inv_max - inv_min)).expand(BV, D, 1, 1)
        cand = inv.expand(BV, D, H, W) if per_pixel else inv.repeat(1, 1, H, W)
        depth = (1.0 / cand).unsqueeze(1).repeat(1, J, 1, 1, 1).reshape(BV * J, D, H, W)
        tgt_in = tgt.reshape(BV * J, C, H, W).clone().requires_grad_(True)
        ref_in = ref.clone().requires_grad_(True)
        warped = mt.warp_with_pose_depth_candidates(tgt_in, ref_k.unsqueeze(1).repeat(1, J, 1, 1).reshape(-1, 3, 3),
                                                    pose.reshape(-1, 4, 4), depth)
        w5 = warped.view(BV, J, C, D, H, W)
        cost = ((ref_in.unsqueeze(-3).unsqueeze(1) * w5).sum(2) / (C ** 0.5)).mean(1)
        gcost = torch.randn(cost.shape, generator=g)
        (cost * gcost).sum().backward()
        out.update({f"{tag}_ref": ref, f"{tag}_tgt": tgt, f"{tag}_intr": ref_k, f"{tag}_pose": pose,
                    f"{tag}_depth": depth.view(BV, J, D, H, W)[:, 0], f"{tag}_warped": w5, f"{tag}_cost": cost,
                    f"{tag}_dcost": gcost, f"{tag}_dref": ref_in.grad, f"{tag}_dtgt": tgt_in.grad.view(BV, J, C, H, W),
                    f"{tag}_feats": torch.stack(feats, 1), f"{tag}_extr": torch.stack(extr, 1)})
    np.savez_compressed(OUT / "cost_volume.npz", **{k: t2n(v) for k, v in out.items()})


def gen_adapter():
    ga = importlib.import_module("src.model.encoder.common.gaussian_adapter")
    gs = importlib.import_module("src.model.encoder.common.gaussians")
    pj = importlib.import_module("src.geometry.projection")
    g = torch.Generator().manual_seed(2)
    B, V, h, w = 1, 2, 6, 8
    ad = ga.GaussianAdapter(ga.GaussianAdapterCfg(1e-10, 3.0, 2))
    ext = torch.eye(4).repeat(B, V, 1, 1)
    ext[:, 1, :3, 3] = torch.tensor([0.1, -0.05, 0.02])
    K = torch.tensor([[1.0, 0, 0.5], [0, 1.2, 0.45], [0, 0, 1]]).repeat(B, V, 1, 1)
    xy, _ = pj.sample_image_grid((h, w))
    coords = xy.reshape(1, 1, h * w, 1, 1, 2) + 0.01 * torch.randn(B, V, h * w, 1, 1, 2, generator=g)
    depths = 1 + 9 * torch.rand(B, V, h * w, 1, 1, generator=g)
    opac = torch.rand(B, V, h * w, 1, 1, generator=g)
    raw = torch.randn(B, V, h * w, 1, 1, ad.d_in, generator=g)
    imgs = torch.rand(B, V, 3, h, w, generator=g)
    e = ext[:, :, None, None, None]
    k = K[:, :, None, None, None]
    res = ad.forward(e, k, coords, depths, opac, raw, (h, w), input_images=imgs)
    q = torch.randn(5, 4, generator=g)
    sc = torch.rand(5, 3, generator=g)
    rays_o, rays_d = pj.get_world_rays(coords, e, k)
    out = {"extrinsics": ext, "intrinsics": K, "coordinates": coords, "depths": depths, "opacities": opac,
           "raw": raw, "images": imgs, "means": res.means, "covariances": res.covariances,
           "harmonics": res.harmonics, "scales": res.scales, "rotations": res.rotations,
           "out_opacities": res.opacities, "quat": q, "scale3": sc, "quat_matrix": gs.quaternion_to_matrix(q),
           "build_cov": gs.build_covariance(sc, q), "rays_o": rays_o, "rays_d": rays_d,
           "fov_K": K[0], "fov": pj.get_fov(K[0]), "grid_xy": xy,
           "grid_ij": pj.sample_image_grid((h, w))[1]}
    np.savez_compressed(OUT / "adapter.npz", **{k: t2n(v) for k, v in out.items()})


def _candidate_block():
    """The depth-candidate lines of MultiViewUniMatch.forward (mv_unimatch.py:416-475), read
    from the reference source at generation time and run as they stand: the class itself
    cannot be built offline (its __init__ fetches DINOv2 through torch.hub)."""
    src = (REF / "src/model/encoder/unimatch/mv_unimatch.py").read_text().splitlines()
    a = next(i for i, ln in enumerate(src) if "num_depth_candidates = self.num_depth_candidates // (4**scale_idx)" in ln)
    b = next(i for i in range(a, len(src)) if "intrinsics_input = torch.stack(intrinsics_curr" in src[i])
    import textwrap
    return compile(textwrap.dedent("\n".join(src[a:b])), "mv_unimatch.py:depth-candidates", "exec")


def gen_matching():
    """batch_features_camera_parameters with an nn_matrix (mv_transformer.py:653-747) and the
    per-scale depth candidates (mv_unimatch.py:416-475) -> matching.npz."""
    mvt = importlib.import_module("src.model.encoder.unimatch.mv_transformer")
    g = torch.Generator().manual_seed(3)
    out = {}
    B, V, C, H, W = 2, 4, 4, 3, 5
    feats = [torch.randn(B, C, H, W, generator=g) for _ in range(V)]
    intr = [torch.rand(B, 3, 3, generator=g) for _ in range(V)]
    extr = [torch.randn(B, 4, 4, generator=g) for _ in range(V)]
    nn = torch.stack([torch.stack([torch.tensor([i] + [(i + k) % V for k in (1, 3)]) for i in range(V)]),
                      torch.stack([torch.tensor([i] + [(i + k) % V for k in (2, 1)]) for i in range(V)])])
    res = mvt.batch_features_camera_parameters(feats, intr, extr, nn_matrix=nn)
    out.update({"nn_feats": torch.stack(feats, 1), "nn_intr": torch.stack(intr, 1), "nn_extr": torch.stack(extr, 1),
                "nn_matrix": nn})
    for k, t in zip(("ref", "ref_k", "ref_e", "tgt", "tgt_k", "tgt_e"), res):
        out[f"nn_{k}"] = t
    code = _candidate_block()
    BV, J, h, w, D = 3, 2, 4, 6, 128
    min_depth = 1.0 / (5 + 5 * torch.rand(BV, generator=g))   # inverse depths, as the caller passes
    max_depth = 1.0 / (0.2 + 0.5 * torch.rand(BV, generator=g))
    for s in (0, 1, 2):
        depth = min_depth.view(-1, 1, 1, 1) + torch.rand(BV, 1, h, w, generator=g) * (max_depth - min_depth).view(-1, 1, 1, 1)
        self = types.SimpleNamespace(num_depth_candidates=D)
        env = {"torch": torch, "self": self, "scale_idx": s, "min_depth": min_depth, "max_depth": max_depth,
               "depth": depth, "features_list_cnn": [torch.zeros(1)], "tgt_features": torch.zeros(BV, J, 1, h, w),
               "h": h, "w": w}
        exec(code, env)
        out[f"cand{s}_depth"] = depth
        out[f"cand{s}_candidates"] = env["depth_candidates"]
        out[f"cand{s}_candidates_curr"] = env["depth_candidates_curr"]
    out["cand_min"], out["cand_max"] = min_depth, max_depth
    np.savez_compressed(OUT / "matching.npz", **{k: t2n(v) for k, v in out.items()})


def gen_matching_tokens():
    """The token-feature branch of batch_features_camera_parameters (mv_transformer.py:706-708:
    features [B, HW, C] per view, nn_matrix gather over "b v -> b v hw c") ->
    matching_tokens.npz. The reference's entry assert (features[0].dim() == 4, :665) rejects
    such features, so this runs under `python -O` (asserts stripped), with no_batch=True (the
    batched return unpacks C, H, W from a 4-D feature)."""
    if not sys.flags.optimize:
        raise SystemExit("matching_tokens: run as `python -O tests/golden/make_golden.py matching_tokens`")
    mvt = importlib.import_module("src.model.encoder.unimatch.mv_transformer")
    g = torch.Generator().manual_seed(4)
    B, V, HW, C = 2, 4, 6, 5
    feats = [torch.randn(B, HW, C, generator=g) for _ in range(V)]
    intr = [torch.rand(B, 3, 3, generator=g) for _ in range(V)]
    extr = [torch.randn(B, 4, 4, generator=g) for _ in range(V)]
    nn = torch.stack([torch.stack([torch.tensor([i] + [(i + k) % V for k in (1, 2)]) for i in range(V)]),
                      torch.stack([torch.tensor([i] + [(i + k) % V for k in (3, 1)]) for i in range(V)])])
    q, qk, qe, kv, kvk, kve = mvt.batch_features_camera_parameters(feats, intr, extr, nn_matrix=nn, no_batch=True)
    out = {"feats": torch.stack(feats, 1), "intr": torch.stack(intr, 1), "extr": torch.stack(extr, 1),
           "nn_matrix": nn}
    for k, lst in zip(("ref", "ref_k", "ref_e", "tgt", "tgt_k", "tgt_e"), (q, qk, qe, kv, kvk, kve)):
        out[k] = torch.stack(lst, 1)  # [B, V, ...] (one entry per reference view)
    np.savez_compressed(OUT / "matching_tokens.npz", **{k: t2n(v) for k, v in out.items()})


def gen_ply():
    """src/model/ply_export.py:26-115 on seeded inputs: export_ply with a non-identity c2w, and
    save_gaussian_ply on a 2-view 20x20 context (the 8-pixel border trim, "h w spp v" order,
    camera -> world rotations). The recorded vertex arrays are stored as float32 [N, 17]
    (columns in construct_list_of_attributes(0) order)."""
    import types as _t
    from scipy.spatial.transform import Rotation
    pe = importlib.import_module("src.model.ply_export")
    rec = importlib.import_module("plyfile").RECORD
    g = torch.Generator().manual_seed(21)
    out = {}

    def c2w_of(euler, t):
        m = torch.eye(4)
        m[:3, :3] = torch.from_numpy(Rotation.from_euler("xyz", euler).as_matrix()).float()
        m[:3, 3] = torch.tensor(t)
        return m

    def unit_q(n):
        q = torch.randn(n, 4, generator=g)
        return q / q.norm(dim=-1, keepdim=True)

    G = 64
    ext = c2w_of([0.3, -0.2, 0.5], [0.1, 0.2, 0.3])
    means = torch.randn(G, 3, generator=g)
    scales = torch.rand(G, 3, generator=g) * 0.1 + 1e-3
    rot = unit_q(G)
    harm = torch.randn(G, 3, 9, generator=g)
    opac = torch.rand(G, generator=g) * 0.98 + 0.01
    rec.clear()
    with tempfile.TemporaryDirectory() as td:
        pe.export_ply(ext, means, scales, rot, harm, opac, Path(td) / "a.ply")
    (_, els), = rec
    (name, data), = els
    assert name == "vertex"
    out.update(export_ext=ext, export_means=means, export_scales=scales, export_rot=rot, export_harm=harm,
               export_opac=opac, export_vertex=np.stack([data[f] for f in data.dtype.names], axis=1))
    v, h, w = 2, 20, 20
    N = v * h * w
    exts = torch.stack([c2w_of([0.1, 0.4, -0.3], [0.0, 0.1, 0.2]), c2w_of([-0.2, 0.1, 0.25], [0.3, -0.1, 0.0])])
    gs = _t.SimpleNamespace(means=torch.randn(1, N, 3, generator=g), harmonics=torch.randn(1, N, 3, 9, generator=g),
                            opacities=torch.rand(1, N, generator=g) * 0.98 + 0.01)
    dump = {"rotations": unit_q(N)[None], "scales": (torch.rand(1, N, 3, generator=g) * 0.1 + 1e-3)}
    example = {"context": {"extrinsics": exts[None], "image": torch.rand(1, v, 3, h, w, generator=g)}}
    rec.clear()
    with tempfile.TemporaryDirectory() as td:
        pe.save_gaussian_ply(gs, dump, example, Path(td) / "b.ply")
    (_, els), = rec
    (_, data), = els
    out.update(save_means=gs.means, save_harm=gs.harmonics, save_opac=gs.opacities, save_rot=dump["rotations"],
               save_scales=dump["scales"], save_ext=exts, save_hw=np.array([v, h, w]),
               save_vertex=np.stack([data[f] for f in data.dtype.names], axis=1))
    np.savez_compressed(OUT / "ply.npz", **{k: t2n(x) for k, x in out.items()})


if __name__ == "__main__":
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    setup_imports()
    torch.set_default_dtype(torch.float32)
    only = sys.argv[1:]  # e.g. `make_golden.py matching` regenerates one fixture file
    for name, fn in (("cuda_splatting", gen_cuda_splatting), ("cost_volume", gen_cost_volume),
                     ("adapter", gen_adapter), ("matching", gen_matching), ("ply", gen_ply)):
        if not only or name in only:
            fn()
    if "matching_tokens" in only:  # separate: needs `python -O` (see gen_matching_tokens)
        gen_matching_tokens()
    for f in sorted(OUT.glob("*.npz")):
        print(f.name, f.stat().st_size)
