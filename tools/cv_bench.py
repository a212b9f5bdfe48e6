"""Time the fused plane-sweep cost volume (dcv_cost_volume_fwd/bwd) against torch
grid_sample + correlation on the same GPU, at SURVEY §8(d) shapes. Prints GB/s and GFLOP/s."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from my_depthsplat_amd.matching import plane_sweep_cost_volume  # noqa: E402


def torch_cost(ref, tgt, K, pose, depth, clamp=1e-3):
    B, J, C, H, W = tgt.shape
    D = depth.shape[1]
    if depth.dim() == 2:
        depth = depth[:, :, None, None].expand(B, D, H, W)
    ys, xs = torch.meshgrid(torch.arange(H, device=ref.device), torch.arange(W, device=ref.device), indexing="ij")
    grid = torch.stack([xs, ys, torch.ones_like(xs)], 0).float().reshape(1, 3, H * W)
    out = 0
    for j in range(J):
        Kj, Pj = K[:, j], pose[:, j]
        rays = torch.inverse(Kj).bmm(grid.expand(B, 3, H * W))
        rot = torch.bmm(Pj[:, :3, :3], rays)
        pts = rot.unsqueeze(2) * depth.reshape(B, 1, D, H * W) + Pj[:, :3, 3:].unsqueeze(-1)
        pix = torch.bmm(Kj, pts.reshape(B, 3, -1)).reshape(B, 3, D, H * W)
        uv = pix[:, :2] / pix[:, 2:].clamp(min=clamp)
        g = torch.stack([2 * uv[:, 0] / (W - 1) - 1, 2 * uv[:, 1] / (H - 1) - 1], -1)
        wp = F.grid_sample(tgt[:, j], g.reshape(B, D * H, W, 2), mode="bilinear", padding_mode="zeros",
                           align_corners=True).reshape(B, C, D, H, W)
        out = out + (ref[:, :, None] * wp).sum(1) / C ** 0.5
    return out / J


def case(B, J, C, H, W, D, per_pixel, dev):
    g = torch.Generator(device=dev).manual_seed(0)
    ref = torch.randn(B, C, H, W, generator=g, device=dev)
    tgt = torch.randn(B, J, C, H, W, generator=g, device=dev)
    K = torch.tensor([[W * 1.0, 0, W / 2], [0, H * 1.0, H / 2], [0, 0, 1]], device=dev).expand(B, J, 3, 3).contiguous()
    pose = torch.eye(4, device=dev).repeat(B, J, 1, 1)
    pose[..., 0, 3] = -0.1
    d = torch.linspace(0.5, 10, D, device=dev)
    depth = d[None, :, None, None].expand(B, D, H, W).contiguous() if per_pixel else d[None].expand(B, D).contiguous()
    return ref, tgt, K, pose, depth


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


SHAPES = {"a": (2, 1, 128, 32, 32, 128, False, "config A (2v, 32^2, C128, D128)"),
          "b0": (2, 1, 128, 64, 64, 128, False, "config B scale 0 (2v, 64^2, C128, D128)"),
          "b1": (2, 1, 64, 128, 128, 32, True, "config B scale 1 (per-pixel D32)"),
          "d0": (6, 2, 128, 56, 96, 128, False, "config D scale 0 (6v, 2 nbrs, 56x96)")}
dev = torch.device("cuda:0")
pick = sys.argv[1:] or ["b0", "b1", "d0"]  # e.g. `python tools/cv_bench.py a` (one shape per profile pass)
for (B, J, C, H, W, D, pp, name) in [SHAPES[k] for k in pick]:
    ref, tgt, K, pose, depth = case(B, J, C, H, W, D, pp, dev)
    hip = plane_sweep_cost_volume(ref, tgt, K, pose, depth)
    tr = torch_cost(ref, tgt, K, pose, depth)
    err = float((hip - tr).abs().max() / tr.abs().max())
    t_h = timeit(lambda: plane_sweep_cost_volume(ref, tgt, K, pose, depth))
    t_t = timeit(lambda: torch_cost(ref, tgt, K, pose, depth), n=5)
    r2 = ref.clone().requires_grad_(True)
    t2 = tgt.clone().requires_grad_(True)
    gcost = torch.randn(B, D, H, W, device=dev)
    t_hb = timeit(lambda: torch.autograd.grad(plane_sweep_cost_volume(r2, t2, K, pose, depth), (r2, t2), gcost))
    flops = 2.0 * B * J * C * D * H * W
    byts = 4.0 * (B * C * H * W * (1 + J) + B * D * H * W + (B * D * H * W if pp else 0))
    print(f"{name}: HIP fwd {t_h * 1e3:8.1f} us ({flops / t_h / 1e6:7.1f} GFLOP/s, {byts / t_h / 1e6:6.1f} GB/s) "
          f"fwd+bwd {t_hb * 1e3:8.1f} us | torch fwd {t_t * 1e3:9.1f} us | max rel err {err:.2e}", flush=True)
