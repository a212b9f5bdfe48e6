"""Time one raster kernel across library variants on the bench workload (GPU box).

usage: python tools/kbench.py [--kernel render_fwd|render_bwd] [--size 256] [--views 3] VARIANT...
VARIANT = name of my_depthsplat_amd/lib/variants/libdsplat_NAME.so, or "main".
Buffers come from one forward (and backward inputs) of the main library; each variant's
entry point is launched on them 200 times between HIP events; outputs are compared with main.
"""
import argparse
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

from my_depthsplat_amd import _lib, raster  # noqa: E402
from my_depthsplat_amd.synthetic import make_scene  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="render_fwd")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--views", type=int, default=3)
    ap.add_argument("--context", type=int, default=2)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    H = W = a.size
    sc = make_scene(batch=1, n_context=a.context, n_targets=a.views, height=H, width=W, seed=1000, device=dev)
    g = sc.gaussians
    V = a.views
    bg = torch.zeros(V, 3, device=dev)
    cams = raster.build_cameras(sc.target_extrinsics[0], sc.target_intrinsics[0], sc.near[0], sc.far[0], bg,
                                [0] * V, True)
    layout = raster.input_layout(g.harmonics, g.covariances, True, True)
    color, state = raster.forward_raw(g.means, g.harmonics, True, 2, g.opacities, g.covariances, cams, V, H, W,
                                      layout)
    G = g.means.shape[1]
    torch.cuda.synchronize()
    print(f"G={G} V={V} {H}x{W} N={int(state.totals[0])}", flush=True)
    st = _lib.stream_of(dev)
    dpix = torch.randn_like(color)
    ref = None
    for name in a.variants:
        path = _lib.LIB_PATH if name == "main" else ROOT / "my_depthsplat_amd/lib/variants" / f"libdsplat_{name}.so"
        lib = ctypes.CDLL(str(path))
        for fn, (res, args) in _lib.SIGNATURES.items():
            f = getattr(lib, fn)
            f.restype, f.argtypes = res, args
        if a.kernel == "render_fwd":
            out = [torch.empty_like(color), torch.empty_like(state.final_T), torch.empty_like(state.n_contrib)]

            def launch():
                return lib.dsr_render_fwd(G, V, H, W, cams.data_ptr(), state.geom.data_ptr(),
                                          state.seg_start.data_ptr(), state.keys.data_ptr(), out[0].data_ptr(),
                                          out[1].data_ptr(), out[2].data_ptr(), st)
        elif a.kernel == "preprocess":
            out = [torch.empty_like(state.geom), torch.empty_like(state.radii),
                   torch.empty(V * state.seg_start.numel(), dtype=torch.int32, device=dev)]

            def launch():
                return lib.dsr_preprocess_fwd(1, G, V, H, W, 2, g.harmonics.shape[-1], g.means.data_ptr(),
                                              g.harmonics.data_ptr(), None, g.opacities.data_ptr(),
                                              g.covariances.data_ptr(), cams.data_ptr(), out[0].data_ptr(),
                                              out[1].data_ptr(), out[2].data_ptr(), layout, st)
        elif a.kernel == "scatter":  # scan + scatter (the scan resets the cursors)
            cur = torch.empty_like(state.seg_start)
            tot = torch.empty(4, dtype=torch.int32, device=dev)
            out = [torch.empty_like(state.keys)]
            seg_count = (state.seg_start[1:] - state.seg_start[:-1]).contiguous()
            ss = torch.empty_like(state.seg_start)

            def launch():
                rc = lib.dsr_bin_scan(V, H, W, seg_count.data_ptr(), ss.data_ptr(), cur.data_ptr(), tot.data_ptr(),
                                      st)
                return rc or lib.dsr_bin_scatter(G, V, H, W, state.geom.data_ptr(), cur.data_ptr(),
                                                 out[0].data_ptr(), st)
        elif a.kernel == "sort":  # copy of the unsorted keys + sort
            cur = torch.empty_like(state.seg_start)
            tot = torch.empty(4, dtype=torch.int32, device=dev)
            seg_count = (state.seg_start[1:] - state.seg_start[:-1]).contiguous()
            ss = torch.empty_like(state.seg_start)
            unsorted = torch.empty_like(state.keys)
            lib.dsr_bin_scan(V, H, W, seg_count.data_ptr(), ss.data_ptr(), cur.data_ptr(), tot.data_ptr(), st)
            lib.dsr_bin_scatter(G, V, H, W, state.geom.data_ptr(), cur.data_ptr(), unsorted.data_ptr(), st)
            out = [torch.empty_like(state.keys)]
            nk = int(state.totals[0])
            maxc = int(state.totals[1])

            def launch():
                out[0][:nk].copy_(unsorted[:nk])
                return lib.dsr_bin_sort(G, V, H, W, state.seg_start.data_ptr(), out[0].data_ptr(), None, maxc, st)
        else:
            out = [torch.zeros_like(state.geom)]

            def launch():
                out[0].zero_()
                return lib.dsr_render_bwd(G, V, H, W, cams.data_ptr(), state.geom.data_ptr(),
                                          state.seg_start.data_ptr(), state.keys.data_ptr(),
                                          state.final_T.data_ptr(), state.n_contrib.data_ptr(), dpix.data_ptr(),
                                          out[0].data_ptr(), st)
        assert launch() == 0, lib.dsplat_last_error()
        torch.cuda.synchronize()
        if ref is None:
            ref = [o.clone() for o in out]
        diff = max(float((o.float() - r.float()).abs().max()) for o, r in zip(out, ref))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(5):
            launch()
        e0.record()
        for _ in range(a.iters):
            launch()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        print(f"{name:>12s}  {a.kernel}  {ms * 1e3:8.2f} us   maxdiff vs first {diff:.3e}", flush=True)


if __name__ == "__main__":
    main()
