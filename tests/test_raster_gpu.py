"""HIP rasterizer vs the CPU oracle (oracle/dsr_oracle.cpp) on the same inputs.

Bars (BASELINE.json north_star): tile/sort indices and preprocess integer outputs
bit-exact; rendered RGB within 1e-4 mean L1 and PSNR delta < 0.01 dB; gradients within
the float32 reordering tolerance written in each test. The oracle itself is "parity
unpinned" against the absent upstream CUDA library (see oracle/dsr_oracle.cpp header).
"""
from __future__ import annotations

import math

import numpy as np
import pytest
import torch

from raster_cases import flat_inputs, oracle_views, packed_cams, scene_inputs, settings_for

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def reference_lists(monkeypatch):
    """Most tests here compare the per-tile lists with the oracle's 3-sigma lists: run the
    stateful path with the reference's binning (raster.STATEFUL_EXACT_BINNING off). The
    product default (exact binning) is covered by test_stateful_exact_binning below and by the
    drop-in module / full-size parity tests."""
    from my_depthsplat_amd import raster
    monkeypatch.setattr(raster, "STATEFUL_EXACT_BINNING", False)


def hip_forward(sc, st, gpu, use_sh=True, bg=(0.0, 0.0, 0.0), need_state=True):
    from my_depthsplat_amd import raster
    means, shs, opac, cov6 = flat_inputs(sc)
    B, v = sc.target_extrinsics.shape[:2]
    view_scene = [i // v for i in range(B * v)]
    cams = packed_cams(st, view_scene, bg).to(gpu)
    feats = shs if use_sh else shs[:, :, 0, :].contiguous()
    deg = math.isqrt(shs.shape[2]) - 1
    h, w = sc.image_shape
    color, state = raster.forward_raw(means.to(gpu), feats.to(gpu), use_sh, deg, opac.to(gpu), cov6.to(gpu), cams,
                                      B * v, h, w, need_state=need_state)
    torch.cuda.synchronize()
    return color, state, cams


def _segments(state, V, T):
    """(begin [V*T], end [V*T], keys): the written, sorted part of each segment, whichever
    layout the forward used (fixed capacity, prefix, depth-cut ends, or bounded segments
    with a spill area: see _spilled)."""
    keys = state.keys.cpu().numpy().view(np.uint64)
    if state.seg_stride == 0:
        start = state.seg_start.cpu().numpy().astype(np.int64)
        return start[:-1], start[1:], keys
    if state.seg_stride == raster_mod().SEG_ENDS:
        return (state.seg_start.cpu().numpy().astype(np.int64)[:-1],
                state.seg_count.cpu().numpy().astype(np.int64), keys)
    cnt = state.seg_count.cpu().numpy().astype(np.int64)
    assert cnt.shape[0] == V * T
    begin = np.arange(V * T, dtype=np.int64) * state.seg_stride
    end = begin + cnt
    sp = _spilled(state, V, T)
    if sp is not None and sp.any():
        # a rebuilt segment's list is in the spill area ([V*T, G] slots), written at least up
        # to the tile's last blended position (what the backward reads): that prefix
        G = state.spill.numel() // (V * T)
        spill = state.spill.view(V * T, G)[torch.from_numpy(np.nonzero(sp)[0]).to(state.spill.device)]
        spill = spill.cpu().numpy().view(np.uint64)
        lim = _tile_max_ncontrib(state, V, T)
        base = len(keys)
        keys = np.concatenate([keys, spill.reshape(-1)])
        for j, sg in enumerate(np.nonzero(sp)[0]):
            begin[sg] = base + j * G
            end[sg] = begin[sg] + min(int(lim[sg]), int(cnt[sg]))
    return begin, end, keys


def _spilled(state, V, T):
    """Bounded segments (training, round 5) that overflowed and were rebuilt: [V*T] bool, or
    None when the state has no spill area. Their _segments part is a prefix of the list."""
    if getattr(state, "spill", None) is None:
        return None
    return state.seg_count.cpu().numpy().astype(np.int64) > state.seg_stride


def _tile_max_ncontrib(state, V, T):
    """Per (view, tile): the largest n_contrib (last blended list position) of its pixels."""
    from my_depthsplat_amd import raster
    nc = state.n_contrib.cpu().numpy().astype(np.int64)
    H, W = nc.shape[1:]
    gx, gy = raster.tiles(H, W)
    assert gx * gy == T
    pad = np.zeros((V, gy * raster.TILE, gx * raster.TILE), np.int64)
    pad[:, :H, :W] = nc
    return pad.reshape(V, gy, raster.TILE, gx, raster.TILE).max(axis=(2, 4)).reshape(V * T)


def _fused_ctx(**options):
    """A RasterContext whose first call already takes the fused sort + composite (a fresh
    context's size hint is the LDS capacity, above FUSED_MAX): hint pinned at 2048 keys."""
    ctx = raster_mod().RasterContext(**options)
    ctx.hints["max_count"] = 2048
    ctx.adapt_hints = False
    return ctx


def raster_mod():
    from my_depthsplat_amd import raster
    return raster


@pytest.mark.parametrize("binning", ["fused", "two_phase"])
@pytest.mark.parametrize("h,w,sh_degree", [(64, 64, 2), (48, 80, 3), (37, 53, 1), (64, 64, 0)])
def test_preprocess_and_binning_bitexact(gpu, h, w, sh_degree, binning, monkeypatch):
    """Both binning layouts: dsr_project_bin (fixed-capacity segments) and the two-phase
    count / scan / scatter path that large problems take (forced by a zero key budget)."""
    from my_depthsplat_amd import raster
    if binning == "two_phase":
        monkeypatch.setattr(raster, "KEY_BUDGET_BYTES", 0)
    sc = scene_inputs(h=h, w=w, sh_degree=sh_degree, seed=1)
    st = settings_for(sc)
    color, state, _ = hip_forward(sc, st, gpu)
    orcs = oracle_views(sc, st)
    geom = state.geom.cpu().numpy()
    radii = state.radii.cpu().numpy()
    gx, gy = (w + 15) // 16, (h + 15) // 16
    T = gx * gy
    begin, end, keys = _segments(state, len(orcs), T)
    for v, o in enumerate(orcs):
        og = o.geom()
        np.testing.assert_array_equal(radii[v], og["radii"])
        vis = og["radii"] > 0
        np.testing.assert_array_equal(geom[v, vis, 0:2], og["xy"][vis])
        np.testing.assert_array_equal(geom[v, vis, 9], og["depth"][vis])
        np.testing.assert_array_equal(geom[v, vis, 2:5], og["conic_opacity"][vis, :3])
        np.testing.assert_array_equal(geom[v, vis, 6:9], og["rgb"][vis])
        okeys, ovals, ranges = o.binning()
        assert int(state.counts[v * T:(v + 1) * T].sum()) == o.num_rendered
        for t in range(T):
            hk = keys[begin[v * T + t]:end[v * T + t]]
            ob, oe = ranges[t]
            # same Gaussians in the same (depth, id) order, same depth bits
            np.testing.assert_array_equal((hk & np.uint64(0xFFFFFFFF)).astype(np.uint32), ovals[ob:oe])
            np.testing.assert_array_equal((hk >> np.uint64(32)).astype(np.uint32),
                                          (okeys[ob:oe] & np.uint64(0xFFFFFFFF)).astype(np.uint32))
        o.close()


def _psnr(a, b):
    mse = float(np.mean((np.clip(a, 0, 1) - np.clip(b, 0, 1)) ** 2))
    return float("inf") if mse == 0 else -10 * math.log10(mse)


@pytest.mark.parametrize("h,w,bg", [(64, 64, (0.0, 0.0, 0.0)), (96, 128, (0.2, 0.5, 1.0))])
def test_render_forward_matches_oracle(gpu, h, w, bg):
    sc = scene_inputs(h=h, w=w, seed=2)
    st = settings_for(sc)
    color, state, _ = hip_forward(sc, st, gpu, bg=bg)
    orcs = oracle_views(sc, st, bg=bg)
    col = color.cpu().numpy()
    ncon = state.n_contrib.cpu().numpy()
    for v, o in enumerate(orcs):
        oc, ot, on = o.image()
        l1 = float(np.abs(col[v] - oc).mean())
        assert l1 < 1e-4, l1
        assert np.abs(col[v] - oc).max() < 1e-3
        p_ref = _psnr(oc, np.zeros_like(oc) + 0.5)
        p_hip = _psnr(col[v], np.zeros_like(oc) + 0.5)
        assert abs(p_ref - p_hip) < 0.01
        assert (ncon[v] == on).mean() > 0.999
        o.close()


def test_colors_precomp_path(gpu):
    sc = scene_inputs(h=48, w=48, seed=3, sh_degree=0)
    st = settings_for(sc)
    color, _, _ = hip_forward(sc, st, gpu, use_sh=False)
    orcs = oracle_views(sc, st, use_sh=False)
    for v, o in enumerate(orcs):
        oc, _, _ = o.image()
        assert float(np.abs(color[v].cpu().numpy() - oc).mean()) < 1e-4
        o.close()


def test_render_backward_matches_oracle(gpu):
    from my_depthsplat_amd import raster
    sc = scene_inputs(h=48, w=64, seed=4, n_tgt=2)
    st = settings_for(sc)
    means, shs, opac, cov6 = flat_inputs(sc)
    B, v = sc.target_extrinsics.shape[:2]
    h, w = sc.image_shape
    color, state, cams = hip_forward(sc, st, gpu)
    g = torch.Generator().manual_seed(7)
    dpix = torch.randn(B * v, 3, h, w, generator=g)
    dmeans, dshs, dopac, dcov6, dm2d, _ = raster.backward_raw(
        means.to(gpu), shs.to(gpu), True, 2, opac.to(gpu), cov6.to(gpu), cams, [i // v for i in range(B * v)], state,
        dpix.to(gpu), want_mean2d=True)
    torch.cuda.synchronize()
    orcs = oracle_views(sc, st)
    acc = {k: 0 for k in ("dmean3D", "dcov6", "dsh", "dopacity")}
    for i, o in enumerate(orcs):
        gr = o.backward(dpix[i].numpy(), f64=True)
        s = float(st["scale"][i])
        acc["dmean3D"] = acc["dmean3D"] + gr["dmean3D"] * s
        acc["dcov6"] = acc["dcov6"] + gr["dcov6"] * (s * s)
        acc["dsh"] = acc["dsh"] + gr["dsh"]
        acc["dopacity"] = acc["dopacity"] + gr["dopacity"]
        np.testing.assert_allclose(dm2d[i].cpu().numpy(), gr["dmean2D"], rtol=5e-4, atol=5e-5 * np.abs(gr["dmean2D"]).max())
        o.close()

    def close(hip, ref, name):
        hip = hip.reshape(ref.shape)
        scale = np.abs(ref).max() + 1e-12
        err = np.abs(hip - ref).max() / scale
        assert err < 5e-4, (name, err)

    close(dmeans[0].cpu().numpy(), acc["dmean3D"], "means")
    close(dcov6[0].cpu().numpy(), acc["dcov6"], "cov6")
    close(dshs[0].cpu().numpy(), acc["dsh"], "sh")
    close(dopac[0].cpu().numpy(), acc["dopacity"], "opacity")


@pytest.mark.parametrize("h,w,seed", [(48, 64, 4), (40, 72, 11)])
def test_render_backward_tile_wave_and_subtile_forms(gpu, monkeypatch, h, w, seed):
    """K7's two forms (round 6): the tile-wave kernel (default; one wave per 16x16 tile, four
    pixels per lane, one dgeom row per (tile, entry)) and the sub-tile-wave kernel
    (DSPLAT_K7_SUBTILE=1). Same skip decisions, different float summation groupings: the
    per-(view, Gaussian) rows and the parameter gradients agree within 1e-4 of their scale, every gradient
    matches the float64 oracle, and each form is bit-identical run to run. 40 x 72: partial
    tiles at the right and bottom edges."""
    from my_depthsplat_amd import raster
    sc = scene_inputs(h=h, w=w, seed=seed, n_tgt=2)
    st = settings_for(sc)
    means, shs, opac, cov6 = flat_inputs(sc)
    B, v = sc.target_extrinsics.shape[:2]
    dpix = torch.randn(B * v, 3, h, w, generator=torch.Generator().manual_seed(9))
    outs = {}
    for form in ("tile", "sub", "tile_again"):
        monkeypatch.setenv("DSPLAT_K7_SUBTILE", "1" if form == "sub" else "0")
        _, state, cams = hip_forward(sc, st, gpu)
        r = raster.backward_raw(means.to(gpu), shs.to(gpu), True, 2, opac.to(gpu), cov6.to(gpu), cams,
                                [i // v for i in range(B * v)], state, dpix.to(gpu), False, want_dgeom=True)
        outs[form] = [t.detach().cpu() for t in (r[0], r[1], r[2], r[3], r[5])]
    for a, b in zip(outs["tile"], outs["tile_again"]):
        assert torch.equal(a, b)
    for a, b, name in zip(outs["tile"], outs["sub"], ("dmeans", "dshs", "dopac", "dcov6", "dgeom")):
        err = float((a - b).abs().max() / (b.abs().max() + 1e-12))
        assert err < 1e-4, (name, err)  # (dcov6: ~3e-5, the conic chain amplifies the regrouping)
    orcs = oracle_views(sc, st)
    acc = {k: 0 for k in ("dmean3D", "dcov6", "dsh", "dopacity")}
    for i, o in enumerate(orcs):
        gr = o.backward(dpix[i].numpy(), f64=True)
        sc_i = float(st["scale"][i])
        acc["dmean3D"] = acc["dmean3D"] + gr["dmean3D"] * sc_i
        acc["dcov6"] = acc["dcov6"] + gr["dcov6"] * (sc_i * sc_i)
        acc["dsh"] = acc["dsh"] + gr["dsh"]
        acc["dopacity"] = acc["dopacity"] + gr["dopacity"]
        o.close()
    for hip, key in zip(outs["tile"][:4], ("dmean3D", "dsh", "dopacity", "dcov6")):
        ref = acc[key]
        err = np.abs(hip[0].numpy().reshape(ref.shape) - ref).max() / (np.abs(ref).max() + 1e-12)
        assert err < 5e-4, (key, err)


def _large_tile_scene(opacity_scale=0.05, constant_opacity=None):
    sc = scene_inputs(h=32, w=32, seed=5, n_ctx=2)
    g = sc.gaussians
    # blow covariances up so every Gaussian covers many tiles; 2 x 32 x 32 = 2048 Gaussians
    # per scene, repeated 6x along G so one tile holds > cap entries
    rep = 6
    g.means = g.means.repeat(1, rep, 1) + 0.001 * torch.arange(rep).repeat_interleave(2048)[None, :, None]
    g.covariances = g.covariances.repeat(1, rep, 1, 1) * 400.0
    g.harmonics = g.harmonics.repeat(1, rep, 1, 1)
    g.opacities = g.opacities.repeat(1, rep) * opacity_scale
    if constant_opacity is not None:
        g.opacities = torch.full_like(g.opacities, constant_opacity)
    return sc


def _check_segments_vs_oracle(state, orcs, V, T):
    """Segment ids vs the oracle's sorted ids: all of them, or with prefix-sorted segments
    the sorted prefix exactly and the unordered tail as a set."""
    begin, end, keys = _segments(state, V, T)
    srt = None if state.seg_sorted is None else state.seg_sorted.cpu().numpy()
    spilled = _spilled(state, V, T)
    for v, o in enumerate(orcs):
        okeys, ovals, ranges = o.binning()
        for t in range(T):
            s = v * T + t
            hk = (keys[begin[s]:end[s]] & np.uint64(0xFFFFFFFF)).astype(np.uint32)
            ob, oe = ranges[t]
            if state.seg_stride == raster_mod().SEG_ENDS or (spilled is not None and spilled[s]):
                # depth cut / rebuilt bounded segment: the head of the sorted list
                assert len(hk) <= oe - ob
                np.testing.assert_array_equal(hk, ovals[ob:ob + len(hk)])
                continue
            if srt is None:
                np.testing.assert_array_equal(hk, ovals[ob:oe])
                continue
            P = int(srt[s])
            assert min(oe - ob, 1024) <= P <= oe - ob
            np.testing.assert_array_equal(hk[:P], ovals[ob:ob + P])
            np.testing.assert_array_equal(np.sort(hk[P:]), np.sort(ovals[ob + P:oe]))


@pytest.mark.parametrize("binning,hint,prefix", [("fused", "low", 4096), ("fused", "exact", 4096),
                                                 ("fused", "exact", 0), ("fused", "between", 0),
                                                 ("fused", "between", 4096), ("two_phase", "exact", 4096),
                                                 ("two_phase", "exact", 0)])
def test_large_tiles_sort_paths(gpu, binning, hint, prefix, monkeypatch):
    """Big Gaussians -> tiles with > LDS-capacity entries. hint = the max-count hint the
    forward sizes the sort with: low -> in-kernel HBM radix path; exact -> MSD split into
    LDS-sized groups; between (above the LDS capacity, below the real maximum) -> split
    launch whose too-large segments fall back to one HBM-sorted group (prefix 0) or are
    prefix-sorted. prefix: raster.SORT_PREFIX (0 = sort every entry)."""
    from my_depthsplat_amd import _lib, raster
    cap = _lib.load().dsr_sort_lds_capacity()
    if binning == "two_phase":
        monkeypatch.setattr(raster, "KEY_BUDGET_BYTES", 0)
        monkeypatch.setattr(raster, "CUT_PREFIX", 0)  # full scatter (the depth cut has its own tests)
    monkeypatch.setattr(raster, "SORT_PREFIX", prefix)
    monkeypatch.setitem(raster.default_context(gpu).hints, "max_count", {"low": 1, "exact": 12288 + 8, "between": cap + 1}[hint])
    monkeypatch.setattr(raster.default_context(gpu), "adapt_hints", False)  # keep the hint fixed
    sc = _large_tile_scene()
    st = settings_for(sc)
    color, state, _ = hip_forward(sc, st, gpu)
    assert state.max_count > cap
    assert (state.seg_sorted is not None) == (prefix > 0 and hint != "low")
    orcs = oracle_views(sc, st)
    _check_segments_vs_oracle(state, orcs, 2, 4)
    ncon = state.n_contrib.cpu().numpy()
    for v, o in enumerate(orcs):
        oc, _, on = o.image()
        assert float(np.abs(color[v].cpu().numpy() - oc).mean()) < 1e-4
        assert (ncon[v] == on).mean() > 0.999
        o.close()


@pytest.mark.parametrize("n_keep", [1900, 2600, 3500, 5000])
def test_sort_render_lds_classes(gpu, n_keep, monkeypatch):
    """dsr_sort_render's LDS classes (2048 / 3072 / 4096 keys per tile, picked by
    max_count_hint) on tiles of ~n_keep entries: below, inside and above each class (above:
    the in-kernel HBM sort). Every class writes the oracle's sorted lists and the same image,
    n_contrib and final T bit for bit."""
    from my_depthsplat_amd import raster
    monkeypatch.setitem(raster.default_context(gpu).hints, "max_count", 4096)  # fused sort + render
    monkeypatch.setattr(raster.default_context(gpu), "adapt_hints", False)
    sc = _large_tile_scene(opacity_scale=0.02)
    g = sc.gaussians
    g.means, g.covariances = g.means[:, :n_keep].contiguous(), g.covariances[:, :n_keep].contiguous()
    g.harmonics, g.opacities = g.harmonics[:, :n_keep].contiguous(), g.opacities[:, :n_keep].contiguous()
    st = settings_for(sc)
    outs = {}
    for hint in (4096, 3072, 2048):
        monkeypatch.setattr(raster, "SORT_RENDER_HINT", hint)
        color, state, _ = hip_forward(sc, st, gpu)
        assert state.seg_stride > 0 and state.seg_sorted is None  # the fused launch ran
        outs[hint] = (color, state.n_contrib.clone(), state.final_T.clone(), _segments(state, 2, 4))
    assert max(int(c) for c in outs[4096][3][1] - outs[4096][3][0]) > 0.8 * n_keep
    for hint in (3072, 2048):
        for a, b in zip(outs[hint][:3], outs[4096][:3]):
            assert torch.equal(a, b), f"class {hint} differs from class 4096"
    b0, e0, k0 = outs[4096][3]
    for hint in (3072, 2048):
        b1, e1, k1 = outs[hint][3]
        for s in range(len(b0)):
            np.testing.assert_array_equal(k1[b1[s]:e1[s]], k0[b0[s]:e0[s]])
    monkeypatch.setattr(raster, "SORT_RENDER_HINT", 2048)
    color, state, _ = hip_forward(sc, st, gpu)
    _check_segments_vs_oracle(state, oracle_views(sc, st), 2, 4)


@pytest.mark.parametrize("binning", ["fused", "two_phase"])
def test_prefix_sort_overflow_fixup(gpu, binning, monkeypatch):
    """Faint Gaussians (alpha just above 1/255): no pixel saturates, so the unsorted tail of
    every long segment would still blend -> each such tile is flagged, sorted in full and
    rendered again. Outputs and gradients must equal those of a full sort, bit for bit."""
    from my_depthsplat_amd import raster
    if binning == "two_phase":
        monkeypatch.setattr(raster, "KEY_BUDGET_BYTES", 0)
        monkeypatch.setattr(raster, "CUT_PREFIX", 0)
    monkeypatch.setitem(raster.default_context(gpu).hints, "max_count", 12288 + 8)
    monkeypatch.setattr(raster.default_context(gpu), "adapt_hints", False)
    sc = _large_tile_scene(constant_opacity=0.0045)
    st = settings_for(sc)
    runs = {}
    for prefix in (4096, 0):
        monkeypatch.setattr(raster, "SORT_PREFIX", prefix)
        color, state, cams = hip_forward(sc, st, gpu)
        runs[prefix] = (color.cpu(), state.final_T.cpu(), state.n_contrib.cpu(), state)
    st4 = runs[4096][3]
    assert st4.seg_overflow is not None
    big = st4.seg_count.cpu() > 4096
    flagged = st4.seg_overflow.cpu()[:-1] != 0  # last word: the any-flag
    assert bool(flagged.any()) and not bool(flagged[~big].any())
    assert int(st4.seg_overflow[-1]) == 1
    assert torch.equal(st4.seg_sorted.cpu()[flagged], st4.seg_count.cpu()[flagged])  # re-sorted in full
    for a, b in zip(runs[4096][:3], runs[0][:3]):
        assert torch.equal(a, b)
    orcs = oracle_views(sc, st)
    _check_segments_vs_oracle(runs[0][3], orcs, 2, 4)
    for v, o in enumerate(orcs):
        oc, _, on = o.image()
        assert float(np.abs(runs[4096][0][v].numpy() - oc).mean()) < 1e-4
        assert (runs[4096][2][v].numpy() == on).mean() > 0.999
        o.close()


def test_prefix_sort_matches_full_sort(gpu, monkeypatch):
    """Default opacities: the sorted prefix suffices (no tile flagged) and forward outputs
    and backward gradients are bit-identical to sorting every entry."""
    from my_depthsplat_amd import raster
    monkeypatch.setitem(raster.default_context(gpu).hints, "max_count", 12288 + 8)
    monkeypatch.setattr(raster.default_context(gpu), "adapt_hints", False)
    sc = _large_tile_scene(opacity_scale=1.0)
    st = settings_for(sc)
    means, shs, opac, cov6 = flat_inputs(sc)
    B, v = sc.target_extrinsics.shape[:2]
    view_scene = [i // v for i in range(B * v)]
    h, w = sc.image_shape
    deg = math.isqrt(shs.shape[2]) - 1
    out = {}
    for prefix in (4096, 0):
        monkeypatch.setattr(raster, "SORT_PREFIX", prefix)
        cams = packed_cams(st, view_scene, (0.0, 0.0, 0.0)).to(gpu)
        args = [t.to(gpu) for t in (means, shs, opac, cov6)]
        color, state = raster.forward_raw(args[0], args[1], True, deg, args[2], args[3], cams, B * v, h, w)
        dcolor = torch.linspace(-1, 1, color.numel(), device=gpu).view_as(color)
        grads = raster.backward_raw(args[0], args[1], True, deg, args[2], args[3], cams, view_scene, state, dcolor,
                                    want_mean2d=True)
        torch.cuda.synchronize()
        out[prefix] = (state, [color.cpu(), state.final_T.cpu(), state.n_contrib.cpu()] +
                       [g.cpu() for g in grads if g is not None])
    st4 = out[4096][0]
    assert st4.seg_sorted is not None
    unsorted_tail = st4.seg_sorted.cpu() < st4.seg_count.cpu()
    assert bool(unsorted_tail.any())  # the prefix sufficed for some long segment
    fa, fb = out[4096][1], out[0][1]
    for a, b in zip(fa[:3], fb[:3]):  # forward: bit-identical
        assert torch.equal(a, b)
    # gradients: the same per-wave partials summed as fixed-point integers (dsr_render_bwd), so
    # the order the partials arrive in no longer matters: bit-identical. (With float atomics
    # the heavy cancellation on this scene - dL/dopacity terms ~350 for sums ~0.1 - made two
    # runs of one layout differ by ~7e-4 of the max.)
    for a, b in zip(fa[3:], fb[3:]):
        assert torch.equal(a, b)


def _forward_backward(sc, st, gpu):
    from my_depthsplat_amd import raster
    means, shs, opac, cov6 = flat_inputs(sc)
    B, v = sc.target_extrinsics.shape[:2]
    view_scene = [i // v for i in range(B * v)]
    h, w = sc.image_shape
    deg = math.isqrt(shs.shape[2]) - 1
    cams = packed_cams(st, view_scene, (0.0, 0.0, 0.0)).to(gpu)
    args = [t.to(gpu) for t in (means, shs, opac, cov6)]
    color, state = raster.forward_raw(args[0], args[1], True, deg, args[2], args[3], cams, B * v, h, w)
    dcolor = torch.linspace(-1, 1, color.numel(), device=gpu).view_as(color)
    grads = raster.backward_raw(args[0], args[1], True, deg, args[2], args[3], cams, view_scene, state, dcolor,
                                want_mean2d=True)
    torch.cuda.synchronize()
    return state, [color.cpu(), state.final_T.cpu(), state.n_contrib.cpu()] + [g.cpu() for g in grads if g is not None]


@pytest.mark.parametrize("opacity", ["default", "faint"])
def test_depth_cut_matches_full_scatter(gpu, opacity, monkeypatch):
    """Two-phase binning with the depth cut (only the nearest ~CUT_PREFIX entries per tile are
    written and sorted) vs the full scatter + full sort: forward outputs bit-identical,
    gradients equal up to float-atomic order, written heads equal to the oracle's sorted
    lists. default: the heads suffice (some tiles keep an unwritten tail, none is flagged);
    faint (alpha just above 1/255, no pixel saturates): every cut tile is flagged, its tail
    appended, the whole list sorted and the tile rendered again."""
    from my_depthsplat_amd import raster
    monkeypatch.setattr(raster, "KEY_BUDGET_BYTES", 0)
    monkeypatch.setattr(raster, "SORT_PREFIX", 0)
    monkeypatch.setitem(raster.default_context(gpu).hints, "two_phase_max", None)  # no short-list hint from earlier tests
    sc = _large_tile_scene(opacity_scale=1.0) if opacity == "default" else _large_tile_scene(constant_opacity=0.0045)
    st = settings_for(sc)
    out = {}
    for cutp in (1024, 0):
        monkeypatch.setattr(raster, "CUT_PREFIX", cutp)
        out[cutp] = _forward_backward(sc, st, gpu)
    stc = out[1024][0]
    assert stc.seg_stride == raster.SEG_ENDS and out[0][0].seg_stride == 0
    written, counts = stc.written().cpu(), stc.counts.cpu().long()
    nseg = counts.numel()  # seg_overflow: tile flags, any-flag, super-block flags
    flagged = stc.seg_overflow.cpu()[:nseg] != 0
    assert bool((written <= counts).all())
    if opacity == "default":
        assert bool((written < counts).any()) and not bool(flagged.any())
        assert int(stc.seg_overflow[nseg]) == 0
    else:
        assert bool(flagged.any()) and int(stc.seg_overflow[nseg]) == 1
        assert bool((stc.seg_overflow[nseg + 1:] != 0).any())
        assert torch.equal(written[flagged], counts[flagged])  # completed and sorted in full
        assert torch.equal(written[~flagged], counts[~flagged])  # tiles the cut kept whole
    fa, fb = out[1024][1], out[0][1]
    for a, b in zip(fa[:3], fb[:3]):  # forward: bit-identical
        assert torch.equal(a, b)
    # gradients: the same per-wave partials summed as fixed-point integers (dsr_render_bwd), so
    # the order the partials arrive in no longer matters: bit-identical. (With float atomics
    # the heavy cancellation on this scene - dL/dopacity terms ~350 for sums ~0.1 - made two
    # runs of one layout differ by ~7e-4 of the max.)
    for a, b in zip(fa[3:], fb[3:]):
        assert torch.equal(a, b)
    orcs = oracle_views(sc, st)
    _check_segments_vs_oracle(stc, orcs, 2, 4)
    for v, o in enumerate(orcs):
        oc, _, on = o.image()
        assert float(np.abs(fa[0][v].numpy() - oc).mean()) < 1e-4
        assert (fa[2][v].numpy() == on).mean() > 0.999
        o.close()


@pytest.mark.parametrize("case", ["too_small", "fits", "short_lists"])
def test_depth_cut_early_scatter(gpu, case, monkeypatch):
    """Round 6: the depth-cut scatter is queued before the host reads N, into keys sized from the
    previous call's N (hint two_phase_n). too_small: the buffer cannot hold N, the queued launch
    does nothing and the pass is re-run at the exact size; fits: the queued pass is the pass;
    short_lists: the cut was planned (long lists last call) but this call's lists are short, so
    the queued pass ran and its cursors / survivor counters are rewound before the full scatter.
    Every case: forward and gradients bit-identical to the synchronous order (no hint)."""
    from my_depthsplat_amd import raster
    monkeypatch.setattr(raster, "KEY_BUDGET_BYTES", 0)
    monkeypatch.setattr(raster, "SORT_PREFIX", 0)
    monkeypatch.setattr(raster, "CUT_PREFIX", 1 << 20 if case == "short_lists" else 1024)
    sc = _large_tile_scene(opacity_scale=1.0)
    st = settings_for(sc)
    hints = raster.default_context(gpu).hints
    out = {}
    for mode in ("sync", case):
        monkeypatch.setitem(hints, "two_phase_max", 1 << 30 if case == "short_lists" else None)
        monkeypatch.setitem(hints, "two_phase_n",
                            {"sync": None, "too_small": 1, "fits": 1 << 26, "short_lists": 1 << 26}[mode])
        state, res = _forward_backward(sc, st, gpu)
        out[mode] = (state.seg_stride, res)
    assert out["sync"][0] == out[case][0] == (0 if case == "short_lists" else raster.SEG_ENDS)
    for a, b in zip(out["sync"][1], out[case][1]):
        assert torch.equal(a, b)


def test_depth_cut_multiview_scene_vs_oracle(gpu, monkeypatch):
    """A scaled-down 6-view scene (6 x 128x224 context -> G = 172K, ~5K entries per tile):
    the two-phase path with the depth cut writes a fraction of the entries, and the images,
    n_contrib and written list heads still match the oracle (and the full scatter exactly)."""
    from my_depthsplat_amd import raster
    monkeypatch.setattr(raster, "KEY_BUDGET_BYTES", 0)
    monkeypatch.setattr(raster, "SORT_PREFIX", 0)
    sc = scene_inputs(h=128, w=224, n_ctx=6, n_tgt=2, seed=21)
    st = settings_for(sc)
    monkeypatch.setattr(raster, "CUT_PREFIX", 0)
    full, _, _ = hip_forward(sc, st, gpu)
    monkeypatch.setattr(raster, "CUT_PREFIX", 1024)
    monkeypatch.setitem(raster.default_context(gpu).hints, "two_phase_max", None)
    color, state, _ = hip_forward(sc, st, gpu)
    assert state.seg_stride == raster.SEG_ENDS
    written, counts = state.written().cpu(), state.counts.cpu().long()
    assert int(written.sum()) < 0.8 * int(counts.sum())  # the cut wrote a fraction of the entries
    assert torch.equal(color.cpu(), full.cpu())
    orcs = oracle_views(sc, st)
    gx, gy = (224 + 15) // 16, (128 + 15) // 16
    _check_segments_vs_oracle(state, orcs, 2, gx * gy)
    ncon = state.n_contrib.cpu().numpy()
    for v, o in enumerate(orcs):
        oc, _, on = o.image()
        assert float(np.abs(color[v].cpu().numpy() - oc).mean()) < 1e-4
        assert (ncon[v] == on).mean() > 0.999
        o.close()


@pytest.mark.parametrize("opacity", ["default", "faint"])
def test_depth_cut_large_rects(gpu, opacity, monkeypatch):
    """Depth cut with Gaussians whose 3-sigma rects cover more than 16 super-blocks (the
    scatter tests those per (Gaussian, super-block) pair and visits only the tiles of the
    super-blocks that pass): 320x320 (5x5 super-blocks of 4x4 tiles), every 50th Gaussian blown
    up over the whole image. Images equal the full scatter's bit for bit and the written heads
    are the oracle's; faint: every cut tile is flagged and completed by the tail pass."""
    from my_depthsplat_amd import raster
    monkeypatch.setattr(raster, "KEY_BUDGET_BYTES", 0)
    monkeypatch.setattr(raster, "SORT_PREFIX", 0)
    sc = scene_inputs(h=320, w=320, n_ctx=2, n_tgt=2, seed=23)
    g = sc.gaussians
    scale = torch.ones_like(g.opacities)
    scale[:, ::50] = 10000.0
    g.covariances = g.covariances * scale[..., None, None]
    if opacity == "faint":
        g.opacities = torch.full_like(g.opacities, 0.0045)
    st = settings_for(sc)
    monkeypatch.setattr(raster, "CUT_PREFIX", 0)
    full, _, _ = hip_forward(sc, st, gpu)
    monkeypatch.setattr(raster, "CUT_PREFIX", 256)
    monkeypatch.setitem(raster.default_context(gpu).hints, "two_phase_max", None)
    color, state, _ = hip_forward(sc, st, gpu)
    assert state.seg_stride == raster.SEG_ENDS
    cut, _, sb = state.cut_plan
    assert sb == 4
    # some rects span more than 16 of the 25 super-blocks
    r = state.radii.cpu()
    assert int((r > 160).sum()) > 0
    written, counts = state.written().cpu(), state.counts.cpu().long()
    nseg = counts.numel()
    flagged = state.seg_overflow.cpu()[:nseg] != 0
    if opacity == "default":
        assert int(written.sum()) < 0.8 * int(counts.sum())
    else:
        assert bool(flagged.any())
        assert torch.equal(written[flagged], counts[flagged])
    assert torch.equal(color.cpu(), full.cpu())
    # no backward: deferred geometry (the scatter passes list their Gaussians, only those are
    # projected in full), including the tail pass's in the faint case
    monkeypatch.setitem(raster.default_context(gpu).hints, "two_phase_max", None)
    lazy, lst, _ = hip_forward(sc, st, gpu, need_state=False)
    assert lst.seg_stride == raster.SEG_ENDS and not lst.geom_complete
    assert torch.equal(lazy.cpu(), full.cpu())
    # the no-backward cut with every record projected by the count pass (the full-record
    # kernel, the fallback for grids too wide for the compact pre-test records): same images
    monkeypatch.setattr(raster, "DEFER_GEOM", False)
    monkeypatch.setitem(raster.default_context(gpu).hints, "two_phase_max", None)
    img, s2, _ = hip_forward(sc, st, gpu, need_state=False)
    assert s2.seg_stride == raster.SEG_ENDS and s2.geom_complete
    assert torch.equal(img.cpu(), full.cpu())
    orcs = oracle_views(sc, st)
    _check_segments_vs_oracle(state, orcs, 2, 20 * 20)
    for o in orcs:
        o.close()


@pytest.mark.parametrize("route", ["unfused_option", "hint_above_fused_max"])
def test_fixed_capacity_unfused_state_forward(gpu, route):
    """Regression (r3 68ffeda: an unbound variable crashed this path): the fixed-capacity
    forward with a backward's state but WITHOUT the fused sort + composite — dsr_bin_sort +
    dsr_render_fwd, taken when the context disables fusion or when the list-length hint is
    above FUSED_MAX — gives the fused path's image, final T and n_contrib bit for bit."""
    from my_depthsplat_amd import raster
    sc = scene_inputs(h=96, w=128, n_ctx=2, n_tgt=2, seed=27)
    st = settings_for(sc)
    means, shs, opac, cov6 = (t.to(gpu) for t in flat_inputs(sc))
    cams = packed_cams(st, [0, 0]).to(gpu)

    def run(ctx):
        color, state = raster.forward_raw(means, shs, True, 2, opac, cov6, cams, 2, 96, 128, ctx=ctx)
        torch.cuda.synchronize()
        return color.cpu(), state.final_T.cpu(), state.n_contrib.cpu(), state
    ref = run(raster.RasterContext())
    if route == "unfused_option":
        ctx = raster.RasterContext(fused_sort_render=False)
    else:
        ctx = raster.RasterContext()
        ctx.hints["max_count"] = raster.FUSED_MAX + 1
        ctx.adapt_hints = False
    got = run(ctx)
    assert got[3].seg_stride > 0 and got[3].keys is not None  # the fixed-capacity layout
    for a, b in zip(ref[:3], got[:3]):
        assert torch.equal(a, b)


def test_deferred_geometry_short_lists(gpu, monkeypatch):
    """The depth cut planned with deferred geometry (no backward) but the lists turn out
    short (the full scatter runs): every record is then projected through the survivor
    lists holding every Gaussian; images equal the stateful path's bit for bit."""
    from my_depthsplat_amd import raster
    monkeypatch.setattr(raster, "KEY_BUDGET_BYTES", 0)
    monkeypatch.setattr(raster, "CUT_PREFIX", 1024)
    sc = scene_inputs(h=96, w=128, n_ctx=2, n_tgt=2, seed=24)
    st = settings_for(sc)
    monkeypatch.setitem(raster.default_context(gpu).hints, "two_phase_max", None)
    full, fst, _ = hip_forward(sc, st, gpu)
    monkeypatch.setitem(raster.default_context(gpu).hints, "two_phase_max", None)
    lazy, lst, _ = hip_forward(sc, st, gpu, need_state=False)
    assert fst.seg_stride == 0 and lst.seg_stride == 0  # lists short: no cut after all
    assert int(lst.counts.max()) <= 2048
    assert torch.equal(lazy, full)
    assert torch.equal(lst.geom, fst.geom)  # every record written


def test_empty_and_culled(gpu):
    """All Gaussians behind the camera -> background only, N = 0."""
    sc = scene_inputs(h=32, w=48, seed=6)
    sc.gaussians.means = sc.gaussians.means * torch.tensor([1.0, 1.0, -1.0])
    st = settings_for(sc)
    color, state, _ = hip_forward(sc, st, gpu, bg=(0.25, 0.5, 0.75))
    assert state.num_rendered == 0
    ref = torch.tensor([0.25, 0.5, 0.75])[None, :, None, None].expand_as(color.cpu())
    assert torch.equal(color.cpu(), ref)


def test_device_cameras_match_reference_settings(gpu):
    """dsr_build_cameras vs the settings the REFERENCE wrapper handed to its rasterizer
    (tests/golden/cuda_splatting_settings.npz)."""
    from pathlib import Path

    from my_depthsplat_amd import raster
    G = np.load(Path(__file__).parent / "golden" / "cuda_splatting_settings.npz")
    T = lambda k: torch.from_numpy(G[k]).to(gpu)  # noqa: E731
    b = G["extrinsics"].shape[0]
    for tag, si in (("si", True), ("ns", False)):
        cams = raster.build_cameras(T("extrinsics"), T("intrinsics"), T("near"), T("far"), T("bg"), list(range(b)),
                                    si).cpu().numpy()
        for i in range(b):
            np.testing.assert_allclose(cams[i, 0:16], G[f"{tag}_view{i}_viewmatrix"].reshape(16), rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(cams[i, 16:32], G[f"{tag}_view{i}_projmatrix"].reshape(16), rtol=1e-5,
                                       atol=1e-5)
            np.testing.assert_allclose(cams[i, 32:35], G[f"{tag}_view{i}_campos"], rtol=1e-6, atol=1e-7)
            if tag == "si":
                np.testing.assert_allclose(cams[i, 35:37], G["si_view%d_tanfov" % i], rtol=1e-6)
                assert cams[i, 41] == np.float32(1) / G["near"][i]
            assert cams[i, 40:41].view(np.int32)[0] == i


def test_render_cuda_end_to_end_vs_oracle(gpu):
    """Reference-signature render_cuda (device cameras, scale-invariant) vs the oracle fed
    the reference wrapper's float32 settings."""
    from my_depthsplat_amd.cuda_splatting import render_cuda
    sc = scene_inputs(h=64, w=96, seed=8, n_tgt=3)
    st = settings_for(sc)
    g = sc.gaussians
    v = sc.target_extrinsics.shape[1]
    rep = lambda t: t.expand(v, *t.shape[1:]).to(gpu)  # noqa: E731
    out = render_cuda(sc.target_extrinsics[0].to(gpu), sc.target_intrinsics[0].to(gpu), sc.near[0].to(gpu),
                      sc.far[0].to(gpu), (64, 96), torch.zeros(v, 3, device=gpu), rep(g.means), rep(g.covariances),
                      rep(g.harmonics), rep(g.opacities)).cpu().numpy()
    for i, o in enumerate(oracle_views(sc, st)):
        ref, _, _ = o.image()
        assert float(np.abs(out[i] - ref).mean()) < 1e-4
        assert abs(_psnr(out[i], ref * 0 + 0.5) - _psnr(ref, ref * 0 + 0.5)) < 0.01
        o.close()


def test_decoder_batched_views(gpu):
    """DecoderSplattingCUDA (B scenes x v views in one call, no repeat) == per-view render_cuda."""
    from my_depthsplat_amd.cuda_splatting import render_cuda
    from my_depthsplat_amd.decoder import DecoderSplattingCUDA, DecoderSplattingCUDACfg
    from my_depthsplat_amd.synthetic import make_scene
    sc = make_scene(batch=2, n_context=2, n_targets=3, height=48, width=64, seed=9, device=gpu)
    dec = DecoderSplattingCUDA(DecoderSplattingCUDACfg("splatting_cuda"), {"background_color": [0.1, 0.2, 0.3]}).to(gpu)
    out = dec(sc.gaussians, sc.target_extrinsics, sc.target_intrinsics, sc.near, sc.far, (48, 64))
    g = sc.gaussians
    for b in range(2):
        rep = lambda t: t[b:b + 1].expand(3, *t.shape[1:])  # noqa: E731
        want = render_cuda(sc.target_extrinsics[b], sc.target_intrinsics[b], sc.near[b], sc.far[b], (48, 64),
                           dec.background_color.expand(3, 3), rep(g.means), rep(g.covariances), rep(g.harmonics),
                           rep(g.opacities))
        assert torch.equal(out.color[b], want)


def test_sort_render_wide_grid_kernel(gpu, monkeypatch):
    """Inference (no n_contrib) on >= 2048 (view, tile) segments takes the 2048-key class at
    5 waves per EU; its images equal the 3072-key class's bit for bit, and view 0 matches the
    oracle (config B scenes, 4 per call: 12 views x 256 tiles)."""
    from my_depthsplat_amd import raster
    from my_depthsplat_amd.decoder import DecoderSplattingCUDA, DecoderSplattingCUDACfg
    from my_depthsplat_amd.synthetic import make_scene
    sc = make_scene(batch=4, n_context=2, n_targets=3, height=256, width=256, seed=21, device=gpu)
    dec = DecoderSplattingCUDA(DecoderSplattingCUDACfg("splatting_cuda"), {"background_color": [0.0, 0.0, 0.0]}).to(gpu)
    outs = {}
    for hint in (2048, 3072, 2048):
        monkeypatch.setattr(raster, "SORT_RENDER_HINT", hint)
        with torch.no_grad():
            outs.setdefault(hint, []).append(
                dec(sc.gaussians, sc.target_extrinsics, sc.target_intrinsics, sc.near, sc.far, (256, 256)).color)
    assert torch.equal(outs[2048][0], outs[3072][0]) and torch.equal(outs[2048][1], outs[3072][0])
    from my_depthsplat_amd.cuda_splatting import _cov6, camera_settings
    from oracle import raster as orc
    g = sc.gaussians
    shs = g.harmonics[0].transpose(-1, -2).contiguous().cpu()
    st = {k: t.cpu().numpy() for k, t in
          camera_settings(sc.target_extrinsics[0], sc.target_intrinsics[0], sc.near[0], sc.far[0]).items()}
    o = orc.render_settings(g.means[0].cpu().numpy(), shs.numpy(), None, g.opacities[0].cpu().numpy(),
                            _cov6(g.covariances[0]).cpu().numpy(), st, 0, np.zeros(3, np.float32), 256, 256, 2)
    ref, _, _ = o.image()
    o.close()
    assert float(np.abs(outs[2048][0][0, 0].cpu().numpy() - ref).mean()) < 1e-4
    # with a backward (n_contrib tracked: the LAST kernels): same image, same gradients bit
    # for bit (the LDS class changes no per-wave partial; fixed-point sums are order-free)
    res = {}
    for hint in (2048, 3072):
        monkeypatch.setattr(raster, "SORT_RENDER_HINT", hint)
        means = sc.gaussians.means.clone().requires_grad_(True)
        gs = type(sc.gaussians)(means, sc.gaussians.covariances, sc.gaussians.harmonics, sc.gaussians.opacities)
        col = dec(gs, sc.target_extrinsics, sc.target_intrinsics, sc.near, sc.far, (256, 256)).color
        (col * torch.linspace(-1, 1, col.numel(), device=gpu).view_as(col)).sum().backward()
        res[hint] = (col.detach(), means.grad)
    assert torch.equal(res[2048][0], res[3072][0]) and torch.equal(res[2048][0], outs[3072][0])
    assert torch.equal(res[2048][1], res[3072][1])


def test_render_bwd_wide_grid_kernel(gpu):
    """dsr_render_bwd on >= 8192 (view, tile) segments runs the 5-waves-per-EU instance: its
    per-view gradients equal those of the narrow instance (the same call on the first 3 views
    only) bit for bit (fixed-point sums: no atomic-order noise), with one fixed-point unit."""
    from my_depthsplat_amd import _lib, raster
    from my_depthsplat_amd.synthetic import make_scene
    V, H, W = 32, 256, 256
    sc = make_scene(batch=1, n_context=2, n_targets=V, height=H, width=W, seed=33, device=gpu)
    g = sc.gaussians
    cams = raster.build_cameras(sc.target_extrinsics[0], sc.target_intrinsics[0], sc.near[0], sc.far[0],
                                torch.zeros(V, 3, device=gpu), [0] * V, True)
    layout = raster.input_layout(g.harmonics, g.covariances, True, True)
    color, st = raster.forward_raw(g.means, g.harmonics, True, 2, g.opacities, g.covariances, cams, V, H, W, layout)
    G = g.means.shape[1]
    gx, gy = raster.tiles(H, W)
    assert V * gx * gy >= 8192
    dpix = torch.randn(color.shape, generator=torch.Generator(device=gpu).manual_seed(3), device=gpu)
    lib, stream = _lib.load(), _lib.stream_of(gpu)
    sp = None if st.seg_start is None else st.seg_start.data_ptr()
    gscale = torch.empty(raster.GRAD_SCALE_BLOCKS, device=gpu)
    _lib.check(lib.dsr_grad_scale(V, H, W, dpix.data_ptr(), gscale.data_ptr(), stream), "dsr_grad_scale")
    out = {}
    for n in (V, 3):
        dq = torch.zeros((n, G, raster.DGEOM_WORDS), dtype=torch.int64, device=gpu)
        _lib.check(lib.dsr_render_bwd(G, n, H, W, cams.data_ptr(), st.geom.data_ptr(), sp, st.seg_count.data_ptr(),
                                      st.seg_stride, st.keys.data_ptr(), None, st.final_T.data_ptr(),
                                      st.n_contrib.data_ptr(), dpix.data_ptr(), gscale.data_ptr(), dq.data_ptr(),
                                      stream), "dsr_render_bwd")
        dgeom = torch.empty((n, G, raster.GEOM_STRIDE), device=gpu)
        _lib.check(lib.dsr_dgeom_to_float(G, n, st.geom.data_ptr(), dq.data_ptr(), gscale.data_ptr(),
                                          None, dgeom.data_ptr(), stream), "dsr_dgeom_to_float")
        out[n] = (dq, dgeom)
    torch.cuda.synchronize()
    assert torch.equal(out[V][0][:3], out[3][0])  # the fixed-point sums, bit for bit
    b = out[3][1]
    for c in range(9):  # every one of the 9 gradient fields is populated
        assert float(b[..., c].abs().max()) > 0, c


@pytest.mark.parametrize("n_ties", [6, 100000, -1])
def test_equal_depth_ties_sorted_by_id(gpu, n_ties):
    """Equal view-space depths: a few tie pairs (insertion fix-up) and a fronto-parallel
    plane where every Gaussian shares one depth (full id-then-depth radix path). Order
    must match the oracle's stable sort (ties in Gaussian-id order) exactly."""
    sc = scene_inputs(h=64, w=64, seed=12)
    m = sc.gaussians.means.clone()
    if n_ties < 0:
        # a dense cluster a few ulps wide plus far outliers: the cluster falls in one bucket
        # of the sort's 16-bit depth window (run > 32 -> full-width fallback passes)
        G = m.shape[1]
        idx = torch.arange(G)
        m[0, :, 2] = 3.0 + 2e-6 * (idx % 40).float()
        far = idx % 10 == 0
        m[0, far, 2] = 3.0 + 37.0 * torch.rand(int(far.sum()), generator=torch.Generator().manual_seed(2))
    elif n_ties >= m.shape[1]:
        m[..., 2] = 3.0
    else:
        g = torch.Generator().manual_seed(1)
        src = torch.randint(0, m.shape[1], (n_ties,), generator=g)
        dst = torch.randint(0, m.shape[1], (n_ties,), generator=g)
        m[0, dst, 2] = m[0, src, 2]
    sc.gaussians.means = m
    st = settings_for(sc)
    color, state, _ = hip_forward(sc, st, gpu)
    orcs = oracle_views(sc, st)
    begin, end, keys = _segments(state, 2, 16)
    for v, o in enumerate(orcs):
        okeys, ovals, ranges = o.binning()
        for t in range(16):
            hk = keys[begin[v * 16 + t]:end[v * 16 + t]]
            ob, oe = ranges[t]
            np.testing.assert_array_equal((hk & np.uint64(0xFFFFFFFF)).astype(np.uint32), ovals[ob:oe])
        oc, _, _ = o.image()
        assert float(np.abs(color[v].cpu().numpy() - oc).mean()) < 1e-4
        o.close()


def test_reference_layout_gradients(gpu):
    """render_views reads harmonics [S,G,3,d_sh] and full covariances in place; its
    gradients must equal the reference path (transpose + triu gather, autograd)."""
    from my_depthsplat_amd import raster
    from my_depthsplat_amd.cuda_splatting import _cov6, render_views
    from my_depthsplat_amd.synthetic import make_scene
    sc = make_scene(batch=1, n_context=2, n_targets=2, height=48, width=64, seed=13, device=gpu)
    g = sc.gaussians
    v = 2
    ext, K = sc.target_extrinsics[0], sc.target_intrinsics[0]
    bg = torch.zeros(v, 3, device=gpu)
    gp = torch.Generator(device=gpu).manual_seed(5)
    dcol = torch.randn(v, 3, 48, 64, device=gpu, generator=gp)

    def grads(fast):
        m = g.means.clone().requires_grad_(True)
        c = g.covariances.clone().requires_grad_(True)
        h = g.harmonics.clone().requires_grad_(True)
        o = g.opacities.clone().requires_grad_(True)
        if fast:
            img = render_views(ext, K, sc.near[0], sc.far[0], (48, 64), bg, m, c, h, o, [0, 0])
        else:
            cams = raster.build_cameras(ext, K, sc.near[0], sc.far[0], bg, [0, 0], True)
            img, _ = raster.rasterize_views(m, h.transpose(-1, -2), o, _cov6(c), cams, [0, 0], use_sh=True,
                                            sh_degree=2, image_height=48, image_width=64)
        (img * dcol).sum().backward()
        return img.detach(), m.grad, c.grad, h.grad, o.grad

    a, b = grads(True), grads(False)
    assert torch.equal(a[0], b[0])
    for x, y, name in zip(a[1:], b[1:], ("means", "cov", "harmonics", "opacities")):
        err = float((x - y).abs().max() / (y.abs().max() + 1e-12))
        assert err < 1e-5, (name, err)
    assert float(a[2][..., 1, 0].abs().max()) == 0.0  # lower triangle gets no gradient


def test_render_bwd_subnormal_opacity_is_finite(gpu, monkeypatch):
    """dL/do is formed as S(h) * (1 / o). Listed Gaussians of subnormal opacity
    (reference 3-sigma lists keep them; 1 / o would be +inf) must give finite gradients — the
    backward's reach test already drops entries below 1/255, and 1 / o is only formed for
    normal o."""
    from my_depthsplat_amd import raster
    from my_depthsplat_amd.cuda_splatting import _cov6
    from my_depthsplat_amd.synthetic import make_scene
    monkeypatch.setattr(raster, "STATEFUL_EXACT_BINNING", False)
    H, W = 48, 64
    sc = make_scene(batch=1, n_context=2, n_targets=2, height=H, width=W, seed=23, device=gpu)
    g = sc.gaussians
    o0 = g.opacities.clone()
    o0[0, ::7] = 1e-40  # subnormal in float32
    assert bool((o0[0, 0] > 0) & (o0[0, 0] < 1.17549435e-38))
    m = g.means.clone().requires_grad_(True)
    o = o0.requires_grad_(True)
    c = _cov6(g.covariances).clone().requires_grad_(True)
    cams = raster.build_cameras(sc.target_extrinsics[0], sc.target_intrinsics[0], sc.near[0], sc.far[0],
                                torch.zeros(2, 3, device=gpu), [0, 0], True)
    img, radii = raster.rasterize_views(m, g.harmonics.transpose(-1, -2).contiguous(), o, c, cams, [0, 0],
                                        use_sh=True, sh_degree=2, image_height=H, image_width=W)
    assert int((radii[:, ::7] > 0).sum()) > 0  # some subnormal-opacity Gaussians are listed
    img.square().sum().backward()
    for t in (m.grad, o.grad, c.grad):
        assert bool(torch.isfinite(t).all())


def test_graph_capture_replay_matches_eager(gpu):
    """The sync-free forward captured into a hipGraph: replays equal eager calls, and
    replays pick up new data written into the captured input buffers."""
    from my_depthsplat_amd.decoder import DecoderSplattingCUDA, DecoderSplattingCUDACfg
    from my_depthsplat_amd.graphs import GraphedCall
    from my_depthsplat_amd.synthetic import make_scene
    sc = make_scene(batch=1, n_context=2, n_targets=3, height=64, width=96, seed=14, device=gpu)
    dec = DecoderSplattingCUDA(DecoderSplattingCUDACfg("splatting_cuda"), {"background_color": [0, 0, 0]}).to(gpu)

    def step():
        with torch.no_grad():
            return dec(sc.gaussians, sc.target_extrinsics, sc.target_intrinsics, sc.near, sc.far, (64, 96))

    eager = step().color.clone()
    g = GraphedCall(step)
    assert torch.equal(g().color, eager)
    # new scene data through the same buffers
    sc2 = make_scene(batch=1, n_context=2, n_targets=3, height=64, width=96, seed=15, device=gpu)
    for name in ("means", "covariances", "harmonics", "opacities"):
        getattr(sc.gaussians, name).copy_(getattr(sc2.gaussians, name))
    want = step().color.clone()
    assert torch.equal(g().color, want)
    assert not torch.equal(want, eager)


def test_two_graphs_on_two_streams(gpu):
    """bench.py's hipgraph2 mode: two captures of the same render, replayed alternately on two
    HIP streams (consecutive scenes overlap). The captures share no buffer (each owns its
    counters and outputs): every replay equals the eager render, and later replays pick up
    new input data through the shared input tensors."""
    from my_depthsplat_amd.decoder import DecoderSplattingCUDA, DecoderSplattingCUDACfg
    from my_depthsplat_amd.graphs import GraphedCall
    from my_depthsplat_amd.synthetic import make_scene
    sc = make_scene(batch=1, n_context=2, n_targets=3, height=64, width=96, seed=16, device=gpu)
    dec = DecoderSplattingCUDA(DecoderSplattingCUDACfg("splatting_cuda"), {"background_color": [0, 0, 0]}).to(gpu)

    def step():
        with torch.no_grad():
            return dec(sc.gaussians, sc.target_extrinsics, sc.target_intrinsics, sc.near, sc.far, (64, 96))

    eager = step().color.clone()
    gs = [GraphedCall(step), GraphedCall(step)]
    lanes = [torch.cuda.Stream(device=gpu), torch.cuda.Stream(device=gpu)]
    torch.cuda.synchronize()
    for i in range(20):
        with torch.cuda.stream(lanes[i & 1]):
            gs[i & 1]()
    torch.cuda.synchronize()
    assert torch.equal(gs[0].out.color, eager) and torch.equal(gs[1].out.color, eager)
    sc2 = make_scene(batch=1, n_context=2, n_targets=3, height=64, width=96, seed=17, device=gpu)
    for name in ("means", "covariances", "harmonics", "opacities"):
        getattr(sc.gaussians, name).copy_(getattr(sc2.gaussians, name))
    want = step().color.clone()
    torch.cuda.synchronize()
    for i in range(4):
        with torch.cuda.stream(lanes[i & 1]):
            gs[i & 1]()
    torch.cuda.synchronize()
    assert torch.equal(gs[0].out.color, want) and torch.equal(gs[1].out.color, want)


def test_inference_fast_path_matches_state_path(gpu):
    """Eager inference (no grad): cameras built inside the binning kernel by one wave, counters
    re-zeroed by the fused sort + composite and reused by the next call. Repeated calls with
    alternating sizes must keep matching the stateful path (device cameras in double), and the
    in-kernel camera block must match dsr_build_cameras."""
    from my_depthsplat_amd import raster
    from my_depthsplat_amd.cuda_splatting import _cov6, render_views
    from my_depthsplat_amd.synthetic import make_scene
    scenes = {hw: make_scene(batch=1, n_context=2, n_targets=3, height=hw[0], width=hw[1], seed=21, device=gpu)
              for hw in ((48, 64), (64, 96))}
    refs = {}
    for hw, sc in scenes.items():
        g = sc.gaussians
        bg = torch.rand(3, 3, device=gpu)
        cams = raster.build_cameras(sc.target_extrinsics[0], sc.target_intrinsics[0], sc.near[0], sc.far[0], bg,
                                    [0, 0, 0], True)
        img, _ = raster.rasterize_views(g.means, g.harmonics.transpose(-1, -2), g.opacities, _cov6(g.covariances),
                                        cams, [0, 0, 0], use_sh=True, sh_degree=2, image_height=hw[0],
                                        image_width=hw[1])
        refs[hw] = (img, bg, cams)
    for hw in ((48, 64), (64, 96), (48, 64), (48, 64), (64, 96)):
        sc, (ref, bg, cams_ref) = scenes[hw], refs[hw]
        g = sc.gaussians
        with torch.no_grad():
            img = render_views(sc.target_extrinsics[0], sc.target_intrinsics[0], sc.near[0], sc.far[0], hw, bg,
                               g.means, g.covariances, g.harmonics, g.opacities, [0, 0, 0])
        torch.cuda.synchronize()
        assert float((img - ref).abs().mean()) < 1e-5, hw
        assert float((img - ref).abs().max()) < 2e-2, hw
    # camera block of the fast path (the last call's state keeps it) vs the double-precision one
    ci = raster.camera_inputs(sc.target_extrinsics[0], sc.target_intrinsics[0], sc.near[0], sc.far[0], bg,
                              [0, 0, 0], True)
    with torch.no_grad():
        _, st = raster.forward_raw(g.means, g.harmonics, True, 2, g.opacities, g.covariances, ci, 3, hw[0], hw[1],
                                   raster.input_layout(g.harmonics, g.covariances, True, True), need_state=False)
    torch.cuda.synchronize()
    assert st.seg_count is None  # the two-launch path ran (counters consumed)
    c_fast, c_ref = st.cams.view(3, -1)[:, :42], cams_ref.view(3, -1)[:, :42]
    assert torch.allclose(c_fast, c_ref, rtol=1e-5, atol=1e-5), float((c_fast - c_ref).abs().max())
    assert torch.equal(st.cams.view(3, -1)[:, 42:], cams_ref.view(3, -1)[:, 42:])


@pytest.mark.parametrize("cov_scale", [1.0, 30.0, 100.0])
def test_emit_pair_cache_and_overflow(gpu, cov_scale):
    """k_project_emit keeps each count-pass pair (tile, rank, owner) in LDS, 768 per wave, and
    emits keys from that list; a workgroup with a wave over the cap re-expands its rects
    instead. Growing the Gaussians moves workgroups from the first path to the second (both
    occur at 30x); the segments must equal the oracle's sorted lists either way."""
    from my_depthsplat_amd import raster
    sc = scene_inputs(h=128, w=128, seed=7, n_ctx=2)
    sc.gaussians.covariances = sc.gaussians.covariances * cov_scale
    st = settings_for(sc)
    color, state, _ = hip_forward(sc, st, gpu)
    assert state.seg_stride > 0  # fixed-capacity binning (the kernel under test)
    B, v = sc.target_extrinsics.shape[:2]
    gx, gy = raster.tiles(128, 128)
    orcs = oracle_views(sc, st)
    _check_segments_vs_oracle(state, orcs, B * v, gx * gy)
    for i, o in enumerate(orcs):
        oc, _, _ = o.image()
        assert float(np.abs(color[i].cpu().numpy() - oc).mean()) < 1e-4
        o.close()


@pytest.mark.parametrize("case", ["ragged", "culled", "one_view"])
def test_inference_fast_path_edge_cases(gpu, case):
    """The two-launch inference path on a ragged image (50x70: partial edge tiles), a scene
    whose Gaussians are all behind the camera (background only), and a single view; each
    against the stateful path with device cameras, called twice (counters reused)."""
    from my_depthsplat_amd import raster
    from my_depthsplat_amd.cuda_splatting import _cov6, render_views
    from my_depthsplat_amd.synthetic import make_scene
    h, w = (50, 70) if case == "ragged" else (48, 64)
    n_tgt = 1 if case == "one_view" else 2
    sc = make_scene(batch=1, n_context=2, n_targets=n_tgt, height=h, width=w, seed=23, device=gpu)
    g = sc.gaussians
    if case == "culled":
        g.means = g.means * torch.tensor([1.0, 1.0, -1.0], device=gpu)
    vs = [0] * n_tgt
    bg = torch.tensor([[0.25, 0.5, 0.75]], device=gpu).expand(n_tgt, 3).contiguous()
    cams = raster.build_cameras(sc.target_extrinsics[0], sc.target_intrinsics[0], sc.near[0], sc.far[0], bg, vs, True)
    ref, _ = raster.rasterize_views(g.means, g.harmonics.transpose(-1, -2), g.opacities, _cov6(g.covariances), cams,
                                    vs, use_sh=True, sh_degree=2, image_height=h, image_width=w)
    for _ in range(2):
        with torch.no_grad():
            img = render_views(sc.target_extrinsics[0], sc.target_intrinsics[0], sc.near[0], sc.far[0], (h, w), bg,
                               g.means, g.covariances, g.harmonics, g.opacities, vs)
        torch.cuda.synchronize()
        assert img.shape == (n_tgt, 3, h, w)
        assert float((img - ref).abs().mean()) < 1e-5
        if case == "culled":
            want = bg[:, :, None, None].expand_as(img)
            assert torch.equal(img, want)


@pytest.mark.parametrize("case", ["large", "anisotropic", "low_opacity"])
def test_inference_exact_tile_binning(gpu, case):
    """The inference binning (k_project_emit with in-kernel cameras) keeps a (Gaussian, tile)
    pair only when the Gaussian's alpha >= 1/255 ellipse reaches a pixel centre of the tile
    (opacity-aware box, then the exact conic minimum over the tile); the stateful path keeps
    the reference's 3-sigma rects. Dropped pairs never blend, so the images must agree on
    Gaussians that are large, strongly anisotropic, or near / below the 1/255 opacity floor."""
    from my_depthsplat_amd import raster
    from my_depthsplat_amd.cuda_splatting import _cov6, render_views
    from my_depthsplat_amd.synthetic import make_scene
    h, w = 64, 96
    sc = make_scene(batch=1, n_context=2, n_targets=2, height=h, width=w, seed=29, device=gpu)
    g = sc.gaussians
    gen = torch.Generator(device="cpu").manual_seed(5)
    if case == "large":
        g.covariances = g.covariances * 30.0
    elif case == "anisotropic":
        s = torch.tensor([6.0, 0.15, 1.0], device=gpu)
        g.covariances = g.covariances * 20.0 * s[:, None] * s[None, :]
    else:
        u = torch.rand(g.opacities.shape, generator=gen).to(gpu)
        g.opacities = torch.where(u < 0.3, torch.full_like(u, 0.5 / 255.0),
                                  torch.where(u < 0.6, torch.full_like(u, 1.5 / 255.0), g.opacities))
        g.covariances = g.covariances * 10.0
    vs = [0, 0]
    bg = torch.tensor([[0.1, 0.2, 0.3]], device=gpu).expand(2, 3).contiguous()
    cams = raster.build_cameras(sc.target_extrinsics[0], sc.target_intrinsics[0], sc.near[0], sc.far[0], bg, vs, True)
    ref, _ = raster.rasterize_views(g.means, g.harmonics.transpose(-1, -2), g.opacities, _cov6(g.covariances), cams,
                                    vs, use_sh=True, sh_degree=2, image_height=h, image_width=w)
    with torch.no_grad():
        img = render_views(sc.target_extrinsics[0], sc.target_intrinsics[0], sc.near[0], sc.far[0], (h, w), bg,
                           g.means, g.covariances, g.harmonics, g.opacities, vs)
    torch.cuda.synchronize()
    assert float((img - ref).abs().mean()) < 1e-5, case
    assert float((img - ref).abs().max()) < 2e-2, case


@pytest.mark.parametrize("layout", ["fixed", "two_phase"])
@pytest.mark.parametrize("case", ["default", "large", "anisotropic", "low_opacity"])
def test_stateful_exact_binning(gpu, layout, case, monkeypatch):
    """The stateful (training) path with exact tile binning (DSR_LAYOUT_EXACT_BINNING: the
    product default) against the same forward + backward on the reference's 3-sigma lists:
    every exact list is an order-preserving subsequence of the reference list, the images and
    final T are bit-identical (dropped pairs fail the alpha >= 1/255 test at every pixel of
    their tile), and the gradients are bit-identical (a dropped pair is never active at any
    pixel, so every per-wave partial is unchanged, and the fixed-point sums do not depend on
    the order they arrive in). Both key layouts: the
    fixed-capacity dsr_project_bin and the two-phase preprocess / scan / scatter."""
    from my_depthsplat_amd import raster
    sc = scene_inputs(h=64, w=96, seed=31, n_tgt=2)
    g = sc.gaussians
    if case == "large":
        g.covariances = g.covariances * 30.0
    elif case == "anisotropic":
        sv = torch.tensor([6.0, 0.15, 1.0])
        g.covariances = g.covariances * 20.0 * sv[:, None] * sv[None, :]
    elif case == "low_opacity":
        u = torch.rand(g.opacities.shape, generator=torch.Generator().manual_seed(5))
        g.opacities = torch.where(u < 0.3, torch.full_like(u, 0.5 / 255.0),
                                  torch.where(u < 0.6, torch.full_like(u, 1.5 / 255.0), g.opacities))
        g.covariances = g.covariances * 10.0
    st = settings_for(sc)
    if layout == "two_phase":
        monkeypatch.setattr(raster, "KEY_BUDGET_BYTES", 0)
        monkeypatch.setattr(raster, "CUT_PREFIX", 0)
    means, shs, opac, cov6 = flat_inputs(sc)
    B, v = sc.target_extrinsics.shape[:2]
    h, w = sc.image_shape
    gx, gy = raster.tiles(h, w)
    T = gx * gy
    dpix = torch.randn(B * v, 3, h, w, generator=torch.Generator().manual_seed(9)).to(gpu)
    runs = {}
    for exact in (False, True):
        monkeypatch.setattr(raster, "STATEFUL_EXACT_BINNING", exact)
        color, state, cams = hip_forward(sc, st, gpu)
        assert state.pruned_lists == exact
        assert (state.seg_stride > 0) == (layout == "fixed")
        grads = raster.backward_raw(means.to(gpu), shs.to(gpu), True, 2, opac.to(gpu), cov6.to(gpu), cams,
                                    [i // v for i in range(B * v)], state, dpix, want_mean2d=True)
        torch.cuda.synchronize()
        runs[exact] = (color, state, grads)
    (c0, s0, g0), (c1, s1, g1) = runs[False], runs[True]
    assert torch.equal(c1, c0) and torch.equal(s1.final_T, s0.final_T)
    b0, e0, k0 = _segments(s0, B * v, T)
    b1, e1, k1 = _segments(s1, B * v, T)
    n0, n1 = int((e0 - b0).sum()), int((e1 - b1).sum())
    assert n1 <= n0
    if case != "default":
        assert n1 < n0  # something was dropped
    # long two-phase segments are prefix-sorted (seg_sorted: the nearest >= 1024 entries in
    # order, the tail unordered): compare as sets, and the sorted parts for order
    p0 = None if s0.seg_sorted is None else s0.seg_sorted.cpu().numpy()
    p1 = None if s1.seg_sorted is None else s1.seg_sorted.cpu().numpy()
    # bounded segments (the product's training layout) that overflowed keep the sorted list up
    # to the tile's last blended entry: where either run has one, compare those prefixes (the
    # deepest last-blended Gaussian is the same in both lists)
    sp0, sp1 = _spilled(s0, B * v, T), _spilled(s1, B * v, T)
    lim0, lim1 = _tile_max_ncontrib(s0, B * v, T), _tile_max_ncontrib(s1, B * v, T)
    for sg in range(B * v * T):
        ref = k0[b0[sg]:e0[sg]]
        sub = k1[b1[sg]:e1[sg]]
        if (sp0 is not None and sp0[sg]) or (sp1 is not None and sp1[sg]):
            ref, sub = ref[:lim0[sg]], sub[:lim1[sg]]
        assert np.isin(sub, ref).all(), sg
        n_sorted = len(sub) if p1 is None else int(p1[sg])
        assert np.all(sub[1:n_sorted] > sub[:n_sorted - 1]), sg  # keys are distinct
        if p0 is None and p1 is None:  # both fully sorted: sub keeps ref's order
            keep = np.isin(ref, sub)
            assert np.array_equal(ref[keep], sub), sg
    for a, b_, name in zip(g1, g0, ("means", "shs", "opacity", "cov6", "mean2d")):
        if a is None:
            continue
        assert torch.equal(a, b_), (case, layout, name, float((a - b_).abs().max()))


@pytest.mark.parametrize("opacity", [0.012, 0.5])
def test_inference_long_lists_camera_block_vs_stateful(gpu, opacity, monkeypatch):
    """Tiles of > 512 entries through the inference fast path (k_project_emit in camera-block
    mode + the fused k_sort_render without n_contrib) against the stateful exact-binning
    forward fed the same camera block (k_sort_render with n_contrib and sorted keys written
    back): large faint Gaussians whose pixels never saturate (opacity 0.012: T stays ~0.3, every
    walk runs to the end of its list) or saturate early (0.5). Bit-identical images, and the
    oracle within the usual bar."""
    from my_depthsplat_amd import raster
    sc = scene_inputs(h=32, w=32, seed=41, n_ctx=2)
    g = sc.gaussians
    g.covariances = g.covariances * 100.0
    g.opacities = torch.full_like(g.opacities, opacity)
    st = settings_for(sc)
    monkeypatch.setattr(raster, "STATEFUL_EXACT_BINNING", True)
    color_ref, state, cams = hip_forward(sc, st, gpu)
    B, v = sc.target_extrinsics.shape[:2]
    h, w = sc.image_shape
    gx, gy = raster.tiles(h, w)
    b0, e0, _ = _segments(state, B * v, gx * gy)
    lens = e0 - b0
    assert 512 < lens.max() <= 2048  # G = 2 x 32 x 32: every list fits the smallest LDS class
    ncon = state.n_contrib.cpu().numpy()
    if opacity < 0.02:
        assert ncon.max() > 512  # walks run past the first 512 entries
    means, shs, opac, cov6 = flat_inputs(sc)
    with torch.no_grad():
        color, _ = raster.forward_raw(means.to(gpu), shs.to(gpu), True, 2, opac.to(gpu), cov6.to(gpu),
                                      raster.CameraBlock(cams), B * v, h, w,
                                      raster.input_layout(shs, cov6, True, False), need_state=False)
    torch.cuda.synchronize()
    assert torch.equal(color, color_ref)
    for i, o in enumerate(oracle_views(sc, st)):
        oc, _, _ = o.image()
        assert float(np.abs(color[i].cpu().numpy() - oc).mean()) < 1e-4
        o.close()


def test_bounded_training_segments_match_unbounded(gpu):
    """Round 5: forwards with a backward use bounded fixed-capacity segments (RasterContext
    seg_capacity, like the inference fast path). Images, final T and gradients equal the
    G-slot layout's bit for bit — also with a capacity far below the longest tile list, where
    the forward renders the overflowing tiles exactly (rebuilt, their sorted lists stored in
    the spill area) and the backward reads those lists from there."""
    from my_depthsplat_amd import raster
    from my_depthsplat_amd.cuda_splatting import _cov6
    from my_depthsplat_amd.synthetic import make_scene
    H, W = 64, 96
    sc = make_scene(batch=2, n_context=2, n_targets=2, height=H, width=W, seed=31, device=gpu)
    dcol = torch.randn(4, 3, H, W, device=gpu, generator=torch.Generator(device=gpu).manual_seed(2))

    def run(ctx):
        g = sc.gaussians
        m = g.means.clone().requires_grad_(True)
        h = g.harmonics.clone().requires_grad_(True)
        o = g.opacities.clone().requires_grad_(True)
        c = _cov6(g.covariances).clone().requires_grad_(True)
        cams = raster.build_cameras(sc.target_extrinsics.flatten(0, 1), sc.target_intrinsics.flatten(0, 1),
                                    sc.near.flatten(), sc.far.flatten(), torch.zeros(4, 3, device=gpu),
                                    [0, 0, 1, 1], True)
        img, _ = raster.rasterize_views(m, h.transpose(-1, -2), o, c, cams, [0, 0, 1, 1], use_sh=True, sh_degree=2,
                                        image_height=H, image_width=W, ctx=ctx)
        (img * dcol).sum().backward()
        torch.cuda.synchronize()
        return img.detach(), m.grad, h.grad, o.grad, c.grad

    ref = run(_fused_ctx(bounded_train_segments=False))
    for cap in (4096, 64):  # 64: every busy tile overflows (rebuilt, spilled)
        got = run(_fused_ctx(seg_capacity=cap))
        for a, b in zip(got, ref):
            assert torch.equal(a, b), cap


@pytest.mark.parametrize("cap", [4096, 256, 64])
def test_bounded_training_spill_lists(gpu, cap):
    """Bounded training segments, state level: forward_raw + backward_raw with a capacity that
    some tiles (4096) or every tile (256, 64) exceeds, against the G-slot layout on
    large Gaussians. Images, final T, n_contrib and every gradient bit-identical; a segment
    within the capacity holds its full sorted list, a rebuilt one's list in the spill area
    equals the G-slot list up to the tile's last blended entry (all dsr_render_bwd reads)."""
    from my_depthsplat_amd import raster
    sc = scene_inputs(h=64, w=96, seed=31, n_tgt=2, batch=2)
    sc.gaussians.covariances = sc.gaussians.covariances * 30.0
    st = settings_for(sc)
    means, shs, opac, cov6 = (t.to(gpu) for t in flat_inputs(sc))
    B, v = sc.target_extrinsics.shape[:2]
    V, G = B * v, means.shape[1]
    vs = [i // v for i in range(V)]
    cams = packed_cams(st, vs).to(gpu)
    h, w = sc.image_shape
    gx, gy = raster.tiles(h, w)
    T = gx * gy
    dpix = torch.randn(V, 3, h, w, generator=torch.Generator().manual_seed(9)).to(gpu)

    def run(ctx):
        color, state = raster.forward_raw(means, shs, True, 2, opac, cov6, cams, V, h, w, need_state=True, ctx=ctx)
        grads = raster.backward_raw(means, shs, True, 2, opac, cov6, cams, vs, state, dpix, want_mean2d=True)
        torch.cuda.synchronize()
        return color, state, grads

    c0, s0, g0 = run(_fused_ctx(bounded_train_segments=False))
    assert s0.spill is None and s0.seg_stride == G
    c1, s1, g1 = run(_fused_ctx(seg_capacity=cap))
    assert s1.spill is not None and s1.seg_stride == cap
    assert torch.equal(c1, c0) and torch.equal(s1.final_T, s0.final_T) and torch.equal(s1.n_contrib, s0.n_contrib)
    sp = _spilled(s1, V, T)
    cnt = s0.seg_count.cpu().numpy().astype(np.int64)
    assert np.array_equal(sp, cnt > cap)
    assert sp.any()
    if cap == 4096:
        assert not sp.all()
    b0, e0, k0 = _segments(s0, V, T)
    b1, e1, k1 = _segments(s1, V, T)
    lim = _tile_max_ncontrib(s0, V, T)
    for sg in range(V * T):
        ref, got = k0[b0[sg]:e0[sg]], k1[b1[sg]:e1[sg]]
        if sp[sg]:
            assert len(got) == min(int(lim[sg]), len(ref)), sg
            np.testing.assert_array_equal(got, ref[:len(got)])
        else:
            np.testing.assert_array_equal(got, ref)
    for a, b_, name in zip(g1, g0, ("means", "shs", "opacity", "cov6", "mean2d")):
        if a is not None:
            assert torch.equal(a, b_), (cap, name)
