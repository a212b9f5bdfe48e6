"""Depth-cut binning statistics of one render call (configs D / E shapes), on the GPU box.

usage: python tools/cut_case.py {dl3dv,recon12} [--reps N]
Prints entries per tile (all / written by the first scatter), tiles and super-blocks flagged for
the tail pass, and the per-kernel times of the sequence (HIP events on the render stream)."""
import argparse
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def scene(kind, dev, chunk=0):
    from my_depthsplat_amd.synthetic import make_scene, context_cameras, target_cameras
    if kind == "dl3dv":
        H, W, v = 448, 768, 8
        sc = make_scene(batch=1, n_context=6, n_targets=v, height=H, width=W, seed=2000, device=dev)
        return sc.gaussians, sc.target_extrinsics, sc.target_intrinsics, sc.near, sc.far, H, W
    from my_depthsplat_amd.gaussian_adapter import GaussianAdapter, GaussianAdapterCfg, gaussians_from_head
    V, H, W, v = 12, 512, 960, 10
    g = torch.Generator(device=dev).manual_seed(99)
    adapter = GaussianAdapter(GaussianAdapterCfg(1e-10, 3.0, 2)).to(dev)
    head = torch.randn(1, V, H * W, 3 + adapter.d_in, generator=g, device=dev)
    depths = torch.rand(1, V, H * W, 1, 1, generator=g, device=dev) * 9 + 1
    images = torch.rand(1, V, 3, H, W, generator=g, device=dev)
    K = torch.tensor([[1.0, 0, 0.5], [0, 1.0, 0.5], [0, 0, 1]], device=dev)
    ctx = context_cameras(V)[None].to(dev)
    tgt = target_cameras(context_cameras(V), 100)[None, chunk * v:(chunk + 1) * v].to(dev)
    with torch.no_grad():
        gs = gaussians_from_head(head, depths, images, ctx, K.expand(1, V, 3, 3).contiguous(), adapter)
    return (gs, tgt, K.expand(1, v, 3, 3).contiguous(), torch.full((1, v), 0.5, device=dev),
            torch.full((1, v), 100.0, device=dev), H, W)


def scatter_stats(st, V, H, W):
    """What k_scatter_cut's first pass does: Gaussians passing the whole-Gaussian pre-test
    (survivors), the rect tiles they expand, the entries kept; and the tiles expanded if the
    rect were clipped to the bounding box of the super-blocks that pass."""
    cut, _, sb = st.cut_plan
    gx, gy = -(-W // 16), -(-H // 16)
    nsx, nsy = -(-gx // sb), -(-gy // sb)
    geom = st.geom.view(V, -1, 12)
    res = {"sb": sb, "survivors": 0, "visible": 0, "visits": 0, "visits_clipped": 0, "kept": 0}
    for v in range(V):
        rec = geom[v]
        r = rec[:, 10].contiguous().view(torch.int32).long()
        vis = r > 0
        px, py, rr = rec[vis, 0], rec[vis, 1], r[vis].float()
        zb = rec[vis, 9].contiguous().view(torch.int32).long() & 0xFFFFFFFF
        x0 = ((px - rr) / 16).trunc().long().clamp(0, gx)
        y0 = ((py - rr) / 16).trunc().long().clamp(0, gy)
        x1 = ((px + rr + 15) / 16).trunc().long().clamp(0, gx)
        y1 = ((py + rr + 15) / 16).trunc().long().clamp(0, gy)
        ok = (x1 > x0) & (y1 > y0)
        x0, y0, x1, y1, zb = x0[ok], y0[ok], x1[ok], y1[ok], zb[ok]
        sx0, sy0 = x0 // sb, y0 // sb
        sx1, sy1 = (x1 - 1) // sb + 1, (y1 - 1) // sb + 1
        cv = cut[v * nsx * nsy:(v + 1) * nsx * nsy].long() & 0xFFFFFFFF
        small = (sx1 - sx0) * (sy1 - sy0) <= 16
        anyp = torch.zeros_like(small)
        bx0 = torch.full_like(x0, 1 << 30)
        by0 = torch.full_like(x0, 1 << 30)
        bx1 = torch.full_like(x0, -1)
        by1 = torch.full_like(x0, -1)
        kept = torch.zeros_like(x0)
        for dy in range(max(1, int((sy1 - sy0).max()))):
            for dx in range(max(1, int((sx1 - sx0).max()))):
                sx, sy = sx0 + dx, sy0 + dy
                m = (sx < sx1) & (sy < sy1)
                idx = (sy.clamp(max=nsy - 1) * nsx + sx.clamp(max=nsx - 1))
                p = m & (zb <= cv[idx])
                anyp |= p
                bx0 = torch.where(p, torch.minimum(bx0, sx), bx0)
                by0 = torch.where(p, torch.minimum(by0, sy), by0)
                bx1 = torch.where(p, torch.maximum(bx1, sx), bx1)
                by1 = torch.where(p, torch.maximum(by1, sy), by1)
                ox = torch.minimum(x1, sx * sb + sb) - torch.maximum(x0, sx * sb)
                oy = torch.minimum(y1, sy * sb + sb) - torch.maximum(y0, sy * sb)
                kept += torch.where(p, ox.clamp(min=0) * oy.clamp(min=0), 0)
        surv = anyp | ~small
        area = (x1 - x0) * (y1 - y0)
        cx0 = torch.maximum(x0, bx0 * sb)
        cx1 = torch.minimum(x1, bx1 * sb + sb)
        cy0 = torch.maximum(y0, by0 * sb)
        cy1 = torch.minimum(y1, by1 * sb + sb)
        carea = torch.where(anyp, (cx1 - cx0).clamp(min=0) * (cy1 - cy0).clamp(min=0), area)
        res["visible"] += int(ok.sum())
        res["survivors"] += int(surv.sum())
        res["visits"] += int(area[surv].sum())
        res["visits_clipped"] += int(carea[surv].sum())
        res["kept"] += int(kept.sum())
        res["large_rects"] = res.get("large_rects", 0) + int((~small).sum())
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kind", choices=["dl3dv", "recon12"])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--chunk", type=int, default=0, help="recon12: which 10 of the 100 target views")
    a = ap.parse_args()
    from my_depthsplat_amd import raster
    dev = torch.device("cuda:0")
    g, ext, intr, near, far, H, W = scene(a.kind, dev, a.chunk)
    V = ext.shape[1]
    bg = torch.zeros(V, 3, device=dev)
    ci = raster.camera_inputs(ext[0], intr[0], near[0], far[0], bg, [0] * V, True)
    deg = int(round(g.harmonics.shape[-1] ** 0.5)) - 1
    ctx = raster.RasterContext()
    lay = raster.input_layout(g.harmonics, g.covariances, True, True)
    out = {}
    for rep in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.no_grad():
            color, st = raster.forward_raw(g.means, g.harmonics, True, deg, g.opacities, g.covariances, ci, V, H, W,
                                           lay, need_state=False, ctx=ctx)
        torch.cuda.synchronize()
        out[f"wall_ms_{rep}"] = round(1e3 * (time.perf_counter() - t0), 3)
    gx, gy = -(-W // 16), -(-H // 16)
    T = gx * gy
    out["G"], out["V"], out["tiles"] = int(g.means.shape[1]), V, T
    out["stride"] = st.seg_stride
    counts = st.counts.long()
    out["entries_all"] = int(counts.sum())
    out["entries_per_tile_max"] = int(counts.max())
    out["entries_per_tile_mean"] = round(float(counts.float().mean()), 1)
    if st.tile_count is not None:  # depth cut: seg_count = ends after the tail pass
        start = st.seg_start[:-1].long()
        written = st.seg_count.long() - start
        out["entries_written_after_tail"] = int(written.sum())
    if st.seg_overflow is not None:
        ov = st.seg_overflow
        flags = ov[:V * T].view(V, T) != 0
        out["tiles_flagged"] = int(flags.sum())
        out["tiles_flagged_per_view"] = flags.sum(1).tolist()
        if ov.numel() > V * T + 1:
            sbf = ov[V * T + 1:] != 0
            out["superblocks_flagged"] = int(sbf.sum())
            out["superblocks"] = int(sbf.numel())
        out["entries_flagged_tiles"] = int(counts.view(V, T)[flags].sum())
    if st.cut_plan is not None:  # statistics from the full geometry records (no deferral)
        with torch.no_grad():
            _, st2 = raster.forward_raw(g.means, g.harmonics, True, deg, g.opacities, g.covariances, ci, V, H, W, lay,
                                        need_state=False, ctx=raster.RasterContext(defer_geom=False))
        out.update(scatter_stats(st2, V, H, W))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
