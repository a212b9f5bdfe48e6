"""CPU estimate of the epipolar-group band sizes U (distinct tapped positions of the 16
pixels x D depths of a group, extended grid) for a bench cost-volume shape: the MFMA work is
16 x U x C per group against 16 x D x C useful. usage: python tools/cv_band.py TAG"""
import math
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402

tag = sys.argv[1]
ref, tgt, K, pose, depth, (BV, J, C, H, W, D) = bench._costvol_case(tag, torch.device("cpu"), 0)
K, pose, depth = K.double().numpy(), pose.double().numpy(), depth.double().numpy()
b, j = 0, 0
k, P = K[b, j], pose[b, j]
R, t = P[:3, :3], P[:3, 3]
c = -R.T @ t
e = k @ c
ys, xs = np.mgrid[0:H, 0:W]
px, py = xs.ravel().astype(np.float64), ys.ravel().astype(np.float64)
if np.abs(e).sum() < 1e-12:
    key = py
elif abs(e[2]) > 1e-12 and math.hypot(e[0] / e[2] - (W - 1) / 2, e[1] / e[2] - (H - 1) / 2) < 64 * math.hypot(W, H):
    ex, ey = e[0] / e[2], e[1] / e[2]
    v = np.arctan2(py - ey, px - ex)
    v[v < 0] += math.pi
    dmax = max(math.hypot((cc & 1) * (W - 1) - ex, (cc >> 1) * (H - 1) - ey) for cc in range(4))
    nb = min(math.ceil(math.pi * dmax) + 1, 8192)
    key = np.minimum(np.floor(v * nb / math.pi), nb - 1)
else:
    n = math.hypot(e[0], e[1])
    key = np.floor(-e[1] / n * px + e[0] / n * py)
order = np.argsort(key, kind="stable")
kinv = np.linalg.inv(k)
q = kinv @ np.stack([px, py, np.ones_like(px)])
a = k @ (R @ q)
bt = k @ t
Us = []
for g0 in range(0, H * W, 16):
    ids = order[g0:g0 + 16]
    dep = depth[b] if depth.ndim == 2 else depth[b][:, ids // W, ids % W] if depth.ndim == 4 else None
    if depth.ndim == 2:
        dd = np.broadcast_to(dep[:, None], (D, len(ids)))
    else:
        dd = depth[b, :, ids // W, ids % W].reshape(D, len(ids)) if depth.ndim == 3 else depth[b, :, 0][:, ids // W, ids % W]
    xx = a[0, ids] * dd + bt[0]
    yy = a[1, ids] * dd + bt[1]
    zz = np.maximum(a[2, ids] * dd + bt[2], 1e-3)
    ix, iy = xx / zz, yy / zz
    ok = (ix > -1) & (ix < W) & (iy > -1) & (iy < H)
    bx, by = np.floor(ix[ok]).astype(int) + 1, np.floor(iy[ok]).astype(int) + 1
    base = set((by * (W + 2) + bx).tolist())
    taps = set()
    for e_ in base:
        taps.update((e_, e_ + 1, e_ + W + 2, e_ + W + 3))
    Us.append(len(taps))
Us = np.array(Us)
print(f"{tag}: groups={len(Us)} D={D} U mean={Us.mean():.0f} p50={np.median(Us):.0f} p90={np.percentile(Us, 90):.0f} "
      f"max={Us.max()} | MFMA work / useful = {Us.mean() / D:.2f}")
