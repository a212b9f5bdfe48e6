"""Phase timing of k_project_emit (inference binning, in-kernel cameras) from an instrumented
variant (GPU box): per workgroup, s_memrealtime (100 MHz) at start, after projection, after the
count pass, after the global range reservation and at the end of the emission, written into
the tail of the key buffer. usage: python tools/pe_timing_build.py (builds VARIANT "pet"); python tools/pe_timing.py pet [batch]"""
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from my_depthsplat_amd import _lib, raster  # noqa: E402
from my_depthsplat_amd.synthetic import make_scene  # noqa: E402

name = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
H = W = 256
dev = torch.device("cuda:0")
sc = make_scene(batch=B, n_context=2, n_targets=3, height=H, width=W, seed=1000, device=dev)
g = sc.gaussians
V = 3 * B
S, G = g.means.shape[:2]
gx, gy = raster.tiles(H, W)
T = gx * gy
lib = ctypes.CDLL(str(ROOT / "my_depthsplat_amd/lib/variants" / f"libdsplat_{name}.so"))
for fn, (res, args) in _lib.SIGNATURES.items():
    f = getattr(lib, fn)
    f.restype, f.argtypes = res, args
layout = raster.input_layout(g.harmonics, g.covariances, True, True) | raster.LAYOUT_COUNTS_ZEROED
ext = sc.target_extrinsics.reshape(V, 4, 4).contiguous()
K = sc.target_intrinsics.reshape(V, 3, 3).contiguous()
near, far = sc.near.reshape(V).contiguous(), sc.far.reshape(V).contiguous()
bg = torch.zeros(V, 3, device=dev)
vs = torch.arange(B, device=dev, dtype=torch.int32).repeat_interleave(3)
cams = torch.empty((V, raster.CAM_FLOATS), device=dev)
geom = torch.empty((V, G, raster.GEOM_STRIDE), device=dev)
radii = torch.empty((V, G), dtype=torch.int32, device=dev)
cnt = torch.zeros(V * T, dtype=torch.int32, device=dev)
keys = torch.empty(V * T * G, dtype=torch.int64, device=dev)
st = _lib.stream_of(dev)
for _ in range(10):
    cnt.zero_()
    assert lib.dsr_project_bin_cameras(S, G, V, H, W, 2, g.harmonics.shape[-1], g.means.data_ptr(),
                                       g.harmonics.data_ptr(), None, g.opacities.data_ptr(), g.covariances.data_ptr(),
                                       ext.data_ptr(), K.data_ptr(), near.data_ptr(), far.data_ptr(), bg.data_ptr(),
                                       vs.data_ptr(), 1, cams.data_ptr(), geom.data_ptr(), radii.data_ptr(),
                                       cnt.data_ptr(), keys.data_ptr(), layout, st) == 0
torch.cuda.synchronize()
nwg = 8 * ((((G + 255) // 256) * V + 7) // 8)
t = keys[V * T * G - nwg * 8:].view(nwg, 8).cpu().numpy().astype(np.int64)
t = t[t[:, 0] > 0]
base = t[:, 0].min()
us = lambda x: x * 0.01  # noqa: E731
q = lambda a: f"mean={a.mean():6.2f} p10={np.percentile(a, 10):6.2f} p50={np.percentile(a, 50):6.2f} " \
              f"p90={np.percentile(a, 90):6.2f} max={a.max():6.2f}"  # noqa: E731
print(f"{name} B={B}: {len(t)} workgroups, span {us(t[:, 4].max() - base):.2f} us (N={int(cnt.sum())})")
print(f"start        {q(us(t[:, 0] - base))}")
print(f"project      {q(us(t[:, 1] - t[:, 0]))}")
print(f"count pass   {q(us(t[:, 2] - t[:, 1]))}")
print(f"reserve      {q(us(t[:, 3] - t[:, 2]))}")
print(f"emit         {q(us(t[:, 4] - t[:, 3]))}")
print(f"end          {q(us(t[:, 4] - base))}")
print(f"pairs/wg     {q(t[:, 5].astype(float))}")
# residency: workgroups live at once on each CU (HW_ID: CU_ID [11:8], SH_ID [12], SE_ID [15:13];
# XCC_ID [3:0])
hwid, xcc = t[:, 6], t[:, 7]
cu = (xcc & 0xF) * 1000 + ((hwid >> 13) & 7) * 100 + ((hwid >> 12) & 1) * 16 + ((hwid >> 8) & 0xF)
peak = []
for c in np.unique(cu):
    ev = sorted([(s, 1) for s in t[cu == c, 0]] + [(e, -1) for e in t[cu == c, 4]], key=lambda p: (p[0], p[1]))
    live = best = 0
    for _, dlt in ev:
        live += dlt
        best = max(best, live)
    peak.append(best)
peak = np.array(peak)
print(f"CUs used {len(peak)}; workgroups per CU {q(np.bincount(np.searchsorted(np.unique(cu), cu)).astype(float))}")
print(f"max live workgroups per CU {q(peak.astype(float))}")
