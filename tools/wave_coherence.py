"""Per-wave tile coherence of the binning input (6-view 448x768 leg): for each wave of 64
consecutive Gaussians and each target view, the number of (Gaussian, tile) pairs and the
area of the union of their tile rects. Usage (GPU box): python tools/wave_coherence.py"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from my_depthsplat_amd import raster  # noqa: E402
from my_depthsplat_amd.synthetic import make_scene  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    H, W, V = 448, 768, 8
    sc = make_scene(batch=1, n_context=6, n_targets=V, height=H, width=W, seed=2000, device=dev)
    g = sc.gaussians
    cams = raster.build_cameras(sc.target_extrinsics[0], sc.target_intrinsics[0], sc.near[0], sc.far[0],
                                torch.zeros(V, 3, device=dev), [0] * V, True)
    layout = raster.input_layout(g.harmonics, g.covariances, True, True)
    _, state = raster.forward_raw(g.means, g.harmonics, True, 2, g.opacities, g.covariances, cams, V, H, W, layout)
    geom = state.geom  # [V, G, 12]
    px, py = geom[..., 0], geom[..., 1]
    r = geom[..., 10].contiguous().view(torch.int32).float()
    gx, gy = (W + 15) // 16, (H + 15) // 16
    x0 = ((px - r) / 16).floor().clamp(0, gx)
    y0 = ((py - r) / 16).floor().clamp(0, gy)
    x1 = ((px + r + 15) / 16).floor().clamp(0, gx)
    y1 = ((py + r + 15) / 16).floor().clamp(0, gy)
    has = r > 0
    area = torch.where(has, (x1 - x0) * (y1 - y0), torch.zeros_like(r))
    G = geom.shape[1] // 64 * 64
    big = 1e9
    def waves(t, fill, op):
        t = torch.where(has, t, torch.full_like(t, fill))[:, :G].view(V, -1, 64)
        return op(t)
    ux0 = waves(x0, big, lambda t: t.min(-1).values)
    uy0 = waves(y0, big, lambda t: t.min(-1).values)
    ux1 = waves(x1, -1, lambda t: t.max(-1).values)
    uy1 = waves(y1, -1, lambda t: t.max(-1).values)
    tot = area[:, :G].view(V, -1, 64).sum(-1)
    ua = ((ux1 - ux0).clamp(min=0) * (uy1 - uy0).clamp(min=0))
    live = tot > 0
    ratio = (ua[live] / tot[live])
    q = torch.tensor([0.1, 0.5, 0.9, 0.99], device=dev)
    print(f"waves={int(live.sum())} pairs/wave mean={float(tot[live].mean()):.0f} "
          f"union/pairs quantiles={[round(float(v), 3) for v in torch.quantile(ratio, q)]} "
          f"frac(union*16<=pairs)={float((ratio <= 1 / 16).float().mean()):.3f} "
          f"frac(union*4<=pairs)={float((ratio <= 1 / 4).float().mean()):.3f} "
          f"frac(union<=pairs)={float((ratio <= 1).float().mean()):.3f}")
    print(f"radius px mean={float(r[has].mean()):.1f} tiles/gaussian mean={float(area[has].mean()):.1f}")


if __name__ == "__main__":
    main()
