"""Per-tile work of the inference fast path on the bench workload (GPU box): exact-binning
list length per tile and, per 8x8 wave sub-tile, the last list position that blended (how far
compositing walks). usage: python tools/tile_stats.py [H W V]"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from my_depthsplat_amd import raster  # noqa: E402
from my_depthsplat_amd.synthetic import make_scene  # noqa: E402

H, W, V = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (256, 256, 3)
dev = torch.device("cuda:0")
sc = make_scene(batch=1, n_context=2, n_targets=V, height=H, width=W, seed=1000, device=dev)
g = sc.gaussians
bg = torch.zeros(V, 3, device=dev)
layout = raster.input_layout(g.harmonics, g.covariances, True, True)
raster.DEBUG_KEEP_FAST_LISTS = True
raster._spec["max_count"] = 2048  # fused fast path from the first call
ci = raster.camera_inputs(sc.target_extrinsics[0], sc.target_intrinsics[0], sc.near[0], sc.far[0], bg, [0] * V, True)
with torch.no_grad():
    color, st = raster.forward_raw(g.means, g.harmonics, True, 2, g.opacities, g.covariances, ci, V, H, W, layout,
                                   need_state=False)
torch.cuda.synchronize()
cnt = st.seg_count.cpu().numpy().astype(np.int64)
nc = st.n_contrib.cpu().numpy().astype(np.int64).reshape(V, H, W)
gx, gy = (W + 15) // 16, (H + 15) // 16
ncp = np.pad(nc, ((0, 0), (0, gy * 16 - H), (0, gx * 16 - W)))
wmax = ncp.reshape(V, gy, 2, 8, gx, 2, 8).max(axis=(3, 6))            # [V, gy, 2, gx, 2]
tmax = wmax.max(axis=(2, 4)).reshape(-1)
ws = wmax.transpose(0, 1, 3, 2, 4).reshape(-1, 4)
q = lambda a: f"mean={a.mean():.0f} p50={np.percentile(a, 50):.0f} p90={np.percentile(a, 90):.0f} " \
              f"p99={np.percentile(a, 99):.0f} max={a.max()}"
print(f"G={g.means.shape[1]} V={V} {H}x{W} tiles={cnt.size} N={cnt.sum()}")
print(f"entries/tile          {q(cnt)}")
print(f"last blended/tile     {q(tmax)}")
print(f"last blended/wave     {q(ws.reshape(-1))}")
print(f"per-tile wave spread  max/mean={np.mean(ws.max(1) / np.maximum(ws.mean(1), 1)):.2f}")
order = np.argsort(-cnt)[:8]
print("heaviest tiles (n, last):", [(int(cnt[i]), int(tmax[i])) for i in order])

# walk length per wave: the list position at which all 64 pixels of the 8x8 sub-tile have
# stopped (T would fall below 1e-4), the whole list when one never stops
keys = st.keys
geom = st.geom
stride = st.seg_stride
walk = np.zeros((V, gy, 2, gx, 2), np.int64)
never = 0
for vi in range(V):
    gv = geom[vi]
    for ty in range(gy):
        for tx in range(gx):
            s = vi * gx * gy + ty * gx + tx
            n = int(cnt[s])
            ids = (keys[s * stride: s * stride + n] & 0xFFFFFFFF).long()
            rec = gv[ids]
            ys, xs = torch.meshgrid(torch.arange(16, device=dev) + ty * 16, torch.arange(16, device=dev) + tx * 16,
                                    indexing="ij")
            px, py = xs.reshape(-1).float(), ys.reshape(-1).float()
            dx = rec[:, 0][None] - px[:, None]
            dy = rec[:, 1][None] - py[:, None]
            pw = -0.5 * (rec[:, 2][None] * dx * dx + rec[:, 4][None] * dy * dy) - rec[:, 3][None] * dx * dy
            al = torch.clamp(rec[:, 5][None] * torch.exp(pw), max=0.99)
            ok = (pw <= 0) & (al >= 1 / 255)
            f = torch.where(ok, 1 - al, torch.ones_like(al))
            T = torch.cumprod(f.double(), 1)
            stop = T < 1e-4
            has = stop.any(1)
            first = torch.where(has, stop.float().argmax(1), torch.full_like(has, n, dtype=torch.long))
            never += int((~has).sum())
            w = first.reshape(2, 8, 2, 8).amax(dim=(1, 3)).cpu().numpy()
            walk[vi, ty, :, tx, :] = w
walk = walk.reshape(-1)
print(f"walk/wave (exact lists) {q(walk)}; pixels never stopping {never / (V * H * W):.4f}; "
      f"waves walking the whole list {(walk == np.repeat(cnt, 4)).mean():.3f}")
