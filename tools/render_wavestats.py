"""Per-wave work of k_render_fwd (GPU box), from a library built with -DRF_DIAG_WAVESTATS
(python tools/variants.py ws="-DRF_DIAG_WAVESTATS"): wall-clock ticks (100 MHz), chunks of
64 list entries walked and entries composited per wave; plus the segment length.
usage: python tools/render_wavestats.py LIB V H W v"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from my_depthsplat_amd import _lib, raster  # noqa: E402
from my_depthsplat_amd.synthetic import make_scene  # noqa: E402

lib_path = sys.argv[1]
V, H, W, v = (int(x) for x in sys.argv[2:6])
_lib._lib = _lib.load(lib_path)
dev = torch.device("cuda:0")
sc = make_scene(batch=1, n_context=V, n_targets=v, height=H, width=W, seed=1000, device=dev)
g = sc.gaussians
cams = raster.build_cameras(sc.target_extrinsics[0], sc.target_intrinsics[0], sc.near[0], sc.far[0],
                            torch.zeros(v, 3, device=dev), [0] * v, True)
layout = raster.input_layout(g.harmonics, g.covariances, True, True)
for _ in range(3):
    color, st = raster.forward_raw(g.means, g.harmonics, True, 2, g.opacities, g.covariances, cams, v, H, W, layout)
torch.cuda.synchronize()
nc = st.n_contrib.cpu().numpy().astype(np.int64)  # [v, H, W]
gx, gy = W // 16, H // 16
w = nc.reshape(v, gy, 2, 8, gx, 2, 8)  # (view, ty, wy, py, tx, wx, px)
lane0 = w[:, :, :, 0, :, :, 0]
lane1 = w[:, :, :, 0, :, :, 1]
lane2 = w[:, :, :, 0, :, :, 2]
cnt = st.seg_count.cpu().numpy().astype(np.int64).reshape(v, gy, 1, gx, 1)
seglen = np.broadcast_to(cnt, (v, gy, 2, gx, 2))
ticks, chunks, comp, seg = (a.reshape(-1) for a in (lane0, lane1, lane2, seglen))
q = [50, 90, 99, 100]
print(f"waves={ticks.size} ticks(10ns) p50/p90/p99/max={np.percentile(ticks, q).round(0)}")
print(f"chunks walked p50/p90/p99/max={np.percentile(chunks, q).round(0)}  (segment chunks "
      f"p50/max={np.percentile(np.ceil(seg / 64), [50, 100]).round(0)})")
print(f"composited p50/p90/p99/max={np.percentile(comp, q).round(0)}")
full = chunks >= np.ceil(seg / 64)
print(f"waves walking the whole list: {full.mean():.3f}")
top = np.argsort(ticks)[-5:]
for i in top:
    print(f"  slow wave: ticks={ticks[i]} chunks={chunks[i]} composited={comp[i]} seglen={seg[i]}")
print(f"corr(ticks, chunks)={np.corrcoef(ticks, chunks)[0, 1]:.3f} corr(ticks, comp)={np.corrcoef(ticks, comp)[0, 1]:.3f}")
