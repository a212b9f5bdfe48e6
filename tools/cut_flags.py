"""Diagnostic: which tiles the depth cut flags (pixels unsaturated after the written head)
for the config-E reconstruction scene (12-view 512x960, first chunk of 10 target views).
usage (GPU box): python tools/cut_flags.py [--views 10] [--context 12] [--height 512] [--width 960]"""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from my_depthsplat_amd import raster  # noqa: E402
from my_depthsplat_amd.gaussian_adapter import GaussianAdapter, GaussianAdapterCfg, gaussians_from_head  # noqa: E402
from my_depthsplat_amd.synthetic import context_cameras, target_cameras  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--views", type=int, default=10)
ap.add_argument("--context", type=int, default=12)
ap.add_argument("--height", type=int, default=512)
ap.add_argument("--width", type=int, default=960)
ap.add_argument("--targets", type=int, default=100)
ap.add_argument("--first", type=int, default=0)
a = ap.parse_args()
dev = torch.device("cuda:0")
V, H, W, v = a.context, a.height, a.width, a.targets
g = torch.Generator(device=dev).manual_seed(99)
adapter = GaussianAdapter(GaussianAdapterCfg(1e-10, 3.0, 2)).to(dev)
head = torch.randn(1, V, H * W, 3 + adapter.d_in, generator=g, device=dev)
depths = torch.rand(1, V, H * W, 1, 1, generator=g, device=dev) * 9 + 1
images = torch.rand(1, V, 3, H, W, generator=g, device=dev)
K = torch.tensor([[1.0, 0, 0.5], [0, 1.0, 0.5], [0, 0, 1]], device=dev)
gs = gaussians_from_head(head, depths, images, context_cameras(V)[None].to(dev), K.expand(1, V, 3, 3).contiguous(),
                         adapter)
tgt = target_cameras(context_cameras(V), v)[a.first:a.first + a.views].to(dev)
n = tgt.shape[0]
cams = raster.build_cameras(tgt, K.expand(n, 3, 3).contiguous(), torch.full((n,), 0.5, device=dev),
                            torch.full((n,), 100.0, device=dev), torch.zeros(n, 3, device=dev), [0] * n, True)
layout = raster.input_layout(gs.harmonics, gs.covariances, True, True)
with torch.no_grad():
    color, st = raster.forward_raw(gs.means, gs.harmonics, True, 2, gs.opacities, gs.covariances, cams, n, H, W,
                                   layout)
torch.cuda.synchronize()
gx, gy = raster.tiles(H, W)
T = gx * gy
cnt = st.counts.cpu().long()
wr = st.written().cpu()
ov = st.seg_overflow.cpu()[:n * T].bool() if st.seg_overflow is not None else torch.zeros(n * T, dtype=torch.bool)
print(f"N={int(cnt.sum())} per view {int(cnt.sum()) // n}, written {int(wr.sum())} ({float(wr.sum() / cnt.sum()):.3f}), "
      f"flagged tiles {int(ov.sum())} of {n * T}")
ft = torch.nonzero(ov).flatten()
for s in ft[:20].tolist():
    vv, t = divmod(s, T)
    ty, tx = divmod(t, gx)
    fT = st.final_T[vv, ty * 16:(ty + 1) * 16, tx * 16:(tx + 1) * 16].abs()
    print(f"view {vv} tile ({tx},{ty}) count {int(cnt[s])} written {int(wr[s])} final_T max {float(fT.max()):.3g}")
