"""Phase timing of k_sort_render from the instrumented variant built by
tools/sr_timing_build.py (GPU box); the inference launch (2048-key class, no n_contrib).
usage: python tools/sr_timing.py VARIANT [H W V]"""
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
H, W, V = (int(x) for x in sys.argv[2:5]) if len(sys.argv) > 4 else (256, 256, 3)
dev = torch.device("cuda:0")
sc = make_scene(batch=1, n_context=2, n_targets=V, height=H, width=W, seed=1000, device=dev)
g = sc.gaussians
bg = torch.zeros(V, 3, device=dev)
layout = raster.input_layout(g.harmonics, g.covariances, True, True)
raster.DEBUG_KEEP_FAST_LISTS = True
raster._spec["max_count"] = 2048
ci = raster.camera_inputs(sc.target_extrinsics[0], sc.target_intrinsics[0], sc.near[0], sc.far[0], bg, [0] * V, True)
with torch.no_grad():
    color, st = raster.forward_raw(g.means, g.harmonics, True, 2, g.opacities, g.covariances, ci, V, H, W, layout,
                                   need_state=False)
torch.cuda.synchronize()
G = g.means.shape[1]
lib = ctypes.CDLL(str(ROOT / "my_depthsplat_amd/lib/variants" / f"libdsplat_{name}.so"))
for fn, (res, args) in _lib.SIGNATURES.items():
    f = getattr(lib, fn)
    f.restype, f.argtypes = res, args
out = [torch.empty_like(color), torch.empty_like(st.final_T), torch.empty_like(st.n_contrib)]
scr = torch.zeros_like(st.keys)
s = _lib.stream_of(dev)
for _ in range(20):
    assert lib.dsr_sort_render(G, V, H, W, st.cams.data_ptr(), st.geom.data_ptr(), None, st.seg_count.data_ptr(),
                               st.seg_stride, st.keys.data_ptr(), scr.data_ptr(), 0, 0, 2048, out[0].data_ptr(),
                               out[1].data_ptr(), None, s) == 0
torch.cuda.synchronize()
nt = st.seg_count.numel()
t = scr[: nt * 32].view(nt, 4, 8).cpu().numpy().astype(np.int64)
t0, t1, t2, n = t[..., 0], t[..., 1], t[..., 2], t[:, 0, 3] & 0xFFFFFFFF
cf, cc, nch, nent = t[..., 4], t[..., 5], t[..., 6] & 0xFFFFFFFF, t[..., 7]
hwid, xcc = t[:, 0, 3] >> 32, t[:, 0, 6] >> 32
# HW_ID (gfx9): CU_ID [11:8], SH_ID [12], SE_ID [15:13]; XCC_ID [3:0]
cu = (xcc & 0xF) * 1000 + ((hwid >> 13) & 7) * 100 + ((hwid >> 12) & 1) * 16 + ((hwid >> 8) & 0xF)
base = t0.min()
us = lambda x: x * 0.01  # noqa: E731  (100 MHz ticks -> us)
q = lambda a: f"mean={a.mean():6.2f} p10={np.percentile(a, 10):6.2f} p50={np.percentile(a, 50):6.2f} " \
              f"p90={np.percentile(a, 90):6.2f} max={a.max():6.2f}"  # noqa: E731
print(f"{name}: span {us(t2.max() - base):.2f} us over {nt} tiles")
print(f"start         {q(us(t0[:, 0] - base))}")
print(f"sort          {q(us(t1[:, 0] - t0[:, 0]))}")
print(f"composite/wv  {q(us((t2 - t1).reshape(-1)))}")
print(f"tile end      {q(us(t2.max(1) - base))}")
print(f"chunks/wave   {q(nch.reshape(-1).astype(float))}")
print(f"entries/wave  {q(nent.reshape(-1).astype(float))}")
print(f"filter kcyc   {q(cf.reshape(-1) / 1e3)}  per chunk {cf.sum() / max(nch.sum(), 1):.0f} cyc")
print(f"comp kcyc     {q(cc.reshape(-1) / 1e3)}  per entry {cc.sum() / max(nent.sum(), 1):.0f} cyc")
lo, hi = np.argsort(n)[: nt // 10], np.argsort(n)[-nt // 10:]
print(f"sort light/heavy tiles (n {n[lo].mean():.0f} / {n[hi].mean():.0f}): "
      f"{us(t1[lo, 0] - t0[lo, 0]).mean():.2f} / {us(t1[hi, 0] - t0[hi, 0]).mean():.2f} us")

ends = us(t2.max(1) - base)
cus = {}
for i in range(nt):
    cus.setdefault(int(cu[i]), []).append(i)
print(f"{len(cus)} distinct CUs; tiles per CU: {sorted(set(len(v) for v in cus.values()))}")
loads = np.array([n[v].sum() for v in cus.values()])
cu_end = np.array([ends[v].max() for v in cus.values()])
print(f"entries per CU {q(loads.astype(float))}; CU end {q(cu_end)}")
gx = (W + 15) // 16
ex = list(cus.values())[:6]
print("example CU tile sets (seg = view, ty, tx; n):", [[(i // (nt // V), (i % (nt // V)) // gx, i % gx, int(n[i])) for i in v] for v in ex])
