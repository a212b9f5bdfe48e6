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
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--width", type=int, default=0)
    ap.add_argument("--views", type=int, default=3)
    ap.add_argument("--context", type=int, default=2)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--stride", type=int, default=0, help="fused-layout stride override (experiments)")
    ap.add_argument("--two-phase", action="store_true", help="force the two-phase binning layout")
    ap.add_argument("--exact", action="store_true", help="replay the inference path's exact-binning lists")
    ap.add_argument("--no-ncontrib", action="store_true", help="sort_render without n_contrib (inference)")
    ap.add_argument("--hint", type=int, default=0, help="sort_render max_count_hint (LDS class; 0 = largest)")
    ap.add_argument("--counters", action="store_true",
                    help="render_bwd: print the 4 uint32 counters an instrumented variant parks in the padding "
                         "words of dgeom's last two rows")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    H, W = a.height or a.size, a.width or a.size
    sc = make_scene(batch=1, n_context=a.context, n_targets=a.views, height=H, width=W, seed=1000, device=dev)
    g = sc.gaussians
    V = a.views
    bg = torch.zeros(V, 3, device=dev)
    cams = raster.build_cameras(sc.target_extrinsics[0], sc.target_intrinsics[0], sc.near[0], sc.far[0], bg,
                                [0] * V, True)
    layout = raster.input_layout(g.harmonics, g.covariances, True, True)
    if a.two_phase:
        raster.KEY_BUDGET_BYTES = 0
    if a.exact:  # the inference fast path's lists (exact binning), snapshotted for replay
        raster.DEBUG_KEEP_FAST_LISTS = True
        raster._spec["max_count"] = 2048
        ci = raster.camera_inputs(sc.target_extrinsics[0], sc.target_intrinsics[0], sc.near[0], sc.far[0], bg,
                                  [0] * V, True)
        with torch.no_grad():
            color, state = raster.forward_raw(g.means, g.harmonics, True, 2, g.opacities, g.covariances, ci, V, H,
                                              W, layout, need_state=False)
        cams = state.cams
    else:
        color, state = raster.forward_raw(g.means, g.harmonics, True, 2, g.opacities, g.covariances, cams, V, H, W,
                                          layout)
    G = g.means.shape[1]
    GS_ = raster.GEOM_STRIDE
    torch.cuda.synchronize()
    print(f"G={G} V={V} {H}x{W} N={state.num_rendered}", flush=True)
    st = _lib.stream_of(dev)
    dpix = torch.randn_like(color)
    ref = None
    for name in a.variants:
        path = _lib.LIB_PATH if name == "main" else ROOT / "my_depthsplat_amd/lib/variants" / f"libdsplat_{name}.so"
        lib = ctypes.CDLL(str(path))
        for fn, (res, args) in _lib.SIGNATURES.items():
            f = getattr(lib, fn)
            f.restype, f.argtypes = res, args
        sp = None if state.seg_start is None else state.seg_start.data_ptr()
        ws = raster._sort_workspace(lib, V, H, W, state.max_count, dev)
        ws_p = None if ws is None else ws.data_ptr()
        sc_p, stride = state.seg_count.data_ptr(), state.seg_stride
        if a.kernel == "render_fwd":
            out = [torch.empty_like(color), torch.empty_like(state.final_T), torch.empty_like(state.n_contrib)]

            def launch():
                return lib.dsr_render_fwd(G, V, H, W, cams.data_ptr(), state.geom.data_ptr(), sp, sc_p, stride,
                                          state.keys.data_ptr(), None, None, None, out[0].data_ptr(), out[1].data_ptr(),
                                          out[2].data_ptr(), st)
        elif a.kernel in ("project", "project_sort"):  # fused binning (+ sort)
            assert stride > 0, "fused layout expected"
            geom2, radii2 = torch.empty_like(state.geom), torch.empty_like(state.radii)
            cnt2 = torch.empty_like(state.seg_count)
            keys2 = torch.empty_like(state.keys)
            scratch2 = torch.empty_like(state.keys)
            tot2 = torch.empty(4, dtype=torch.int32, device=dev)
            out = [geom2]

            def launch():
                rc = lib.dsr_project_bin(1, G, V, H, W, 2, g.harmonics.shape[-1], g.means.data_ptr(),
                                         g.harmonics.data_ptr(), None, g.opacities.data_ptr(),
                                         g.covariances.data_ptr(), cams.data_ptr(), geom2.data_ptr(),
                                         radii2.data_ptr(), cnt2.data_ptr(), keys2.data_ptr(), layout, st)
                if rc or a.kernel == "project":
                    return rc
                return lib.dsr_bin_sort(G, V, H, W, None, cnt2.data_ptr(), a.stride or G, keys2.data_ptr(),
                                        scratch2.data_ptr(), state.max_count, ws_p, 0, None, None, st)
        elif a.kernel == "project_cam":  # the inference path's binning (in-kernel cameras, exact binning)
            assert stride > 0, "fused layout expected"
            geom2, radii2 = torch.empty_like(state.geom), torch.empty_like(state.radii)
            cnt2 = torch.zeros_like(state.seg_count)
            keys2 = torch.empty_like(state.keys)
            cams2 = torch.empty_like(cams)
            ext, K = sc.target_extrinsics[0].contiguous(), sc.target_intrinsics[0].contiguous()
            near, far = sc.near[0].contiguous(), sc.far[0].contiguous()
            vs = torch.zeros(V, dtype=torch.int32, device=dev)
            out = [geom2]

            def launch():
                cnt2.zero_()
                return lib.dsr_project_bin_cameras(1, G, V, H, W, 2, g.harmonics.shape[-1], g.means.data_ptr(),
                                                   g.harmonics.data_ptr(), None, g.opacities.data_ptr(),
                                                   g.covariances.data_ptr(), ext.data_ptr(), K.data_ptr(),
                                                   near.data_ptr(), far.data_ptr(), bg.data_ptr(), vs.data_ptr(), 1,
                                                   cams2.data_ptr(), geom2.data_ptr(), radii2.data_ptr(),
                                                   cnt2.data_ptr(), keys2.data_ptr(), layout | 4, st)
        elif a.kernel == "sort_render":  # fused sort + composite (keys already sorted: same work)
            assert stride > 0, "fused layout expected"
            out = [torch.empty_like(color), torch.empty_like(state.final_T)]
            if not a.no_ncontrib:
                out.append(torch.empty_like(state.n_contrib))
            scr4 = torch.empty_like(state.keys)

            def launch():
                return lib.dsr_sort_render(G, V, H, W, cams.data_ptr(), state.geom.data_ptr(), None, sc_p, stride,
                                           state.keys.data_ptr(), scr4.data_ptr(), 0, 0, a.hint, out[0].data_ptr(),
                                           out[1].data_ptr(), out[2].data_ptr() if len(out) > 2 else None, st)
        elif a.kernel == "scatter":  # two-phase key scatter from the scan's segment starts
            assert stride == 0, "two-phase layout expected (--two-phase)"
            cur = torch.empty_like(state.seg_start)
            keys3 = torch.empty_like(state.keys)
            out = [state.seg_count]

            def launch():
                cur.copy_(state.seg_start)
                return lib.dsr_bin_scatter(G, V, H, W, state.geom.data_ptr(), cur.data_ptr(), keys3.data_ptr(), 0, st)
        elif a.kernel == "sort_sorted":  # re-sort the (already sorted) keys in place: pass cost only
            tot3 = torch.empty(4, dtype=torch.int32, device=dev)
            scr = torch.empty_like(state.keys)
            out = [state.keys]

            def launch():
                return lib.dsr_bin_sort(G, V, H, W, sp, sc_p, stride, state.keys.data_ptr(), scr.data_ptr(),
                                        state.max_count, ws_p, 0, None, None, st)
        else:
            out = [torch.zeros_like(state.geom)]

            def launch():
                out[0].zero_()
                return lib.dsr_render_bwd(G, V, H, W, cams.data_ptr(), state.geom.data_ptr(), sp, sc_p, stride,
                                          state.keys.data_ptr(), state.final_T.data_ptr(),
                                          state.n_contrib.data_ptr(), dpix.data_ptr(), out[0].data_ptr(), st)
        assert launch() == 0, lib.dsplat_last_error()
        torch.cuda.synchronize()
        if a.counters and a.kernel == "render_bwd":
            flat = out[0].view(-1).view(torch.int32)
            c = [int(flat[-3]), int(flat[-2]), int(flat[-1]), int(flat[-GS_ - 1])]
            print(f"{name:>12s}  counters: entries {c[0]}, entries with an active lane {c[1]}, "
                  f"groups reduced {c[2]} of {c[3]}", flush=True)
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
