"""Per-tile last-contributor positions vs segment sizes (GPU box): how much of each tile's
sorted list the compositing actually consumes. usage: python tools/ncontrib_stats.py V H W v"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from my_depthsplat_amd import raster  # noqa: E402
from my_depthsplat_amd.synthetic import make_scene  # noqa: E402

V, H, W, v = (int(x) for x in sys.argv[1:5])
dev = torch.device("cuda:0")
sc = make_scene(batch=1, n_context=V, n_targets=v, height=H, width=W, seed=2000, device=dev)
g = sc.gaussians
cams = raster.build_cameras(sc.target_extrinsics[0], sc.target_intrinsics[0], sc.near[0], sc.far[0],
                            torch.zeros(v, 3, device=dev), [0] * v, True)
layout = raster.input_layout(g.harmonics, g.covariances, True, True)
color, st = raster.forward_raw(g.means, g.harmonics, True, 2, g.opacities, g.covariances, cams, v, H, W, layout)
torch.cuda.synchronize()
nc = st.n_contrib.cpu().numpy().astype(np.int64)
fT = st.final_T.cpu().numpy()
cnt = st.seg_count.cpu().numpy().astype(np.int64)
gx, gy = (W + 15) // 16, (H + 15) // 16
tmax = np.zeros(v * gy * gx, np.int64)
for vi in range(v):
    t = nc[vi][: gy * 16, : gx * 16] if H % 16 == 0 and W % 16 == 0 else np.pad(nc[vi], ((0, gy * 16 - H), (0, gx * 16 - W)))
    tmax[vi * gx * gy:(vi + 1) * gx * gy] = t.reshape(gy, 16, gx, 16).max(axis=(1, 3)).reshape(-1)
frac = tmax / np.maximum(cnt, 1)
print(f"tiles={tmax.size} entries/tile mean={cnt.mean():.0f} max={cnt.max()} | last contributor per tile: "
      f"mean={tmax.mean():.0f} p90={np.percentile(tmax, 90):.0f} p99={np.percentile(tmax, 99):.0f} max={tmax.max()} | "
      f"fraction of list used: mean={frac.mean():.3f} max={frac.max():.3f} | tiles with last > 4096: "
      f"{(tmax > 4096).mean():.4f}, > 8192: {(tmax > 8192).mean():.4f} | unsaturated pixels "
      f"{(fT > 1e-4 + 1e-7).mean():.4f}")
