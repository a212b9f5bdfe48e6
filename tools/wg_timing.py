"""Per-workgroup timeline of k_sort_render (variant built with -DSR_TIMING, see
tools/variants.py): start / end (s_memrealtime, 100 MHz), tile size and HW placement of every
workgroup at config B. Diagnostics only.
usage: python tools/wg_timing.py [VARIANT]"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from my_depthsplat_amd import _lib, raster  # noqa: E402
from my_depthsplat_amd.synthetic import make_scene  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "srtime"
    lib = _lib.load(ROOT / "my_depthsplat_amd/lib/variants" / f"libdsplat_{name}.so")
    dev = torch.device("cuda:0")
    H = W = 256
    V = 3
    sc = make_scene(batch=1, n_context=2, n_targets=V, height=H, width=W, seed=1000, device=dev)
    g = sc.gaussians
    bg = torch.zeros(V, 3, device=dev)
    cams = raster.build_cameras(sc.target_extrinsics[0], sc.target_intrinsics[0], sc.near[0], sc.far[0], bg,
                                [0] * V, True)
    layout = raster.input_layout(g.harmonics, g.covariances, True, True)
    color, st = raster.forward_raw(g.means, g.harmonics, True, 2, g.opacities, g.covariances, cams, V, H, W, layout)
    G = g.means.shape[1]
    gx, gy = raster.tiles(H, W)
    T = gx * gy
    diag = torch.zeros(4 * V * T + 16, dtype=torch.int64, device=dev)
    out = [torch.empty_like(color), torch.empty_like(st.final_T), torch.empty_like(st.n_contrib)]
    s = _lib.stream_of(dev)
    for it in range(3):
        cnt = st.seg_count.clone()
        rc = lib.dsr_sort_render(G, V, H, W, cams.data_ptr(), st.geom.data_ptr(), None, cnt.data_ptr(), st.seg_stride,
                                 st.keys.data_ptr(), diag.data_ptr(), 0, 0, out[0].data_ptr(), out[1].data_ptr(),
                                 out[2].data_ptr(), s)
        assert rc == 0
    torch.cuda.synchronize()
    d = diag[:4 * V * T].view(V * T, 4).cpu()
    t0, t1, n, hw = d[:, 0], d[:, 1], d[:, 2], d[:, 3]
    base = int(t0.min())
    start, end = (t0 - base).float() * 10e-3, (t1 - base).float() * 10e-3  # us
    dur = end - start
    hwid = hw & 0xFFFFFFFF
    xcc = (hw >> 32) & 0xF
    cu = (hwid >> 8) & 0xF
    sh = (hwid >> 12) & 1
    se = (hwid >> 13) & 0x7
    print(f"kernel span {float(end.max()):.1f} us; start spread {float(start.max()):.1f} us")
    print(f"duration us: mean {float(dur.mean()):.1f} p50 {float(dur.median()):.1f} max {float(dur.max()):.1f}")
    print(f"entries: mean {float(n.float().mean()):.0f} max {int(n.max())}")
    cc = torch.corrcoef(torch.stack([dur, n.float()]))[0, 1]
    print(f"corr(duration, entries) {float(cc):.3f}")
    key = xcc * 1000 + se * 100 + sh * 16 + cu
    uniq, inv = torch.unique(key, return_inverse=True)
    per_cu_end = torch.zeros(len(uniq)).scatter_reduce(0, inv, end, "amax")
    per_cu_n = torch.zeros(len(uniq)).scatter_add(0, inv, n.float())
    per_cu_cnt = torch.zeros(len(uniq)).scatter_add(0, inv, torch.ones_like(end))
    print(f"distinct CUs {len(uniq)}; WGs per CU min {int(per_cu_cnt.min())} max {int(per_cu_cnt.max())}")
    print(f"per-CU entries: mean {float(per_cu_n.mean()):.0f} max {float(per_cu_n.max()):.0f}")
    print(f"per-CU end us: mean {float(per_cu_end.mean()):.1f} max {float(per_cu_end.max()):.1f}")
    print(f"corr(per-CU end, per-CU entries) {float(torch.corrcoef(torch.stack([per_cu_end, per_cu_n]))[0, 1]):.3f}")
    for x in range(8):
        m = xcc == x
        if m.any():
            print(f"  XCC {x}: WGs {int(m.sum())} mean end {float(end[m].mean()):.1f} max end {float(end[m].max()):.1f}"
                  f" mean dur {float(dur[m].mean()):.1f}")
    for v in range(V):
        sl = slice(v * T, (v + 1) * T)
        print(f"  view {v}: mean start {float(start[sl].mean()):.2f} mean end {float(end[sl].mean()):.1f} "
              f"mean entries {float(n[sl].float().mean()):.0f}")
    # within a CU: is the end order the start (dispatch) order?
    order = torch.argsort(end, descending=True)[:8]
    for i in order.tolist():
        v, t = divmod(i, T)
        print(f"  late WG view {v} tile ({t % gx},{t // gx}) start {float(start[i]):.1f} end {float(end[i]):.1f} "
              f"n {int(n[i])} cu-key {int(key[i])}")
    # same tile position across views on the same CU?
    same = sum(1 for t in range(T) if len({int(key[v * T + t]) for v in range(V)}) == 1)
    print(f"tile positions whose {V} views share one CU: {same} of {T}")


if __name__ == "__main__":
    main()
