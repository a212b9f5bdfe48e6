"""Bounded key memory on the inference fast path (dsr_project_bin_cameras seg_capacity).

A segment keeps the first `capacity` entries its tile receives; dsr_sort_render rebuilds a
tile whose count exceeds the capacity from the geometry records and composites it in depth
windows of the LDS class. Images must be bit-identical to the unbounded layout (capacity G)
for every capacity, including tiles longer than one LDS window whose pixels stay live across
windows (faint Gaussians), with exact and with 3-sigma (reference) binning.
"""
import pytest
import torch


def _render(sc, ctx, gpu, H, W):
    from my_depthsplat_amd import raster
    g = sc.gaussians
    V = sc.target_extrinsics.shape[1]
    bg = torch.tensor([[0.2, 0.4, 0.6]], device=gpu).expand(V, 3).contiguous()
    ci = raster.camera_inputs(sc.target_extrinsics[0], sc.target_intrinsics[0], sc.near[0], sc.far[0], bg,
                              [0] * V, True)
    with torch.no_grad():
        color, st = raster.forward_raw(g.means, g.harmonics, True, 2, g.opacities, g.covariances, ci, V, H, W,
                                       raster.input_layout(g.harmonics, g.covariances, True, True),
                                       need_state=False, ctx=ctx)
    torch.cuda.synchronize()
    assert st.seg_count is None, "the fast path (bounded segments) must have run"
    return color, st


def _ctx(gpu, exact, capacity):
    from my_depthsplat_amd import raster
    ctx = raster.RasterContext(exact_binning=exact, seg_capacity=capacity)
    ctx.hints["max_count"] = 2048  # 2048-key LDS class: lists above it span several windows
    ctx.adapt_hints = False
    return ctx


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["plain", "long_faint_rect", "long_faint_exact"])
@pytest.mark.parametrize("capacity", [1, 64, 1000])
def test_bounded_capacity_images_equal_unbounded(gpu, case, capacity):
    from my_depthsplat_amd.synthetic import make_scene
    H = W = 128 if case != "plain" else 96
    sc = make_scene(batch=1, n_context=2, n_targets=3, height=H, width=W, seed=41, device=gpu)
    g = sc.gaussians
    exact = case != "long_faint_rect"
    if case == "long_faint_rect":    # alpha >= 1/255 only near each centre: pixels never saturate
        g.covariances = g.covariances * 200.0
        g.opacities = torch.full_like(g.opacities, 0.0042)
    elif case == "long_faint_exact":
        g.covariances = g.covariances * 400.0
        g.opacities = torch.full_like(g.opacities, 0.006)
    G = g.means.shape[1]
    ref_ctx = _ctx(gpu, exact, G)
    ref, _ = _render(sc, ref_ctx, gpu, H, W)
    ctx = _ctx(gpu, exact, capacity)
    img, st = _render(sc, ctx, gpu, H, W)
    assert st.keys.numel() == 3 * (H // 16) * (W // 16) * capacity  # the bounded allocation
    stats = ctx.last_stats()
    if capacity <= 64:
        assert stats["max_count"] > capacity  # some tiles overflowed and were rebuilt
    assert (stats["rebuilt_tiles"] > 0) == (stats["max_count"] > capacity), stats
    if case != "plain":
        assert stats["max_count"] > 2048, stats  # rebuilt lists span several LDS windows
    assert torch.equal(img, ref), float((img - ref).abs().max())
    # a second call reuses the counters the rebuilt tiles zeroed; with the hints frozen it
    # warns (once) that the first call's tiles went through the slow rebuild
    import warnings
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        img2, _ = _render(sc, ctx, gpu, H, W)
    assert any("frozen segment capacity" in str(w.message) for w in rec) == (stats["rebuilt_tiles"] > 0), \
        [str(w.message) for w in rec]
    assert torch.equal(img2, ref)


def test_automatic_capacity_from_hints():
    """Default capacity: 16384 before any call, then max(4096, 2 x the largest list seen,
    rounded up to a power of two), at most G; the config-B bench shape keeps keys + scratch of
    16 scenes (48 views) under 1 GB instead of 26 GB."""
    from my_depthsplat_amd import raster
    ctx = raster.RasterContext()
    assert ctx.seg_capacity(131072) == 16384
    ctx.hints["max_count"] = 1800
    assert ctx.seg_capacity(131072) == 4096
    ctx.hints["max_count"] = 3000
    assert ctx.seg_capacity(131072) == 8192
    assert ctx.seg_capacity(5000) == 5000
    ctx.hints["max_count"] = 1800
    V, T = 48, 256
    assert 16 * V * T * ctx.seg_capacity(131072) < (1 << 30)


@pytest.mark.gpu
def test_bounded_capacity_under_graph_capture(gpu):
    """A decoder whose capacity is frozen into a hipGraph below its scenes' longest tile lists
    (the rebuild path runs inside the graph): every replay equals an eager render of the
    unbounded layout bit for bit, and the counters the captured sort + composite clears serve
    the next replay."""
    from my_depthsplat_amd.decoder import DecoderSplattingCUDA, DecoderSplattingCUDACfg
    from my_depthsplat_amd.graphs import GraphedCall
    from my_depthsplat_amd.synthetic import make_scene
    H = W = 96
    sc = make_scene(batch=2, n_context=2, n_targets=3, height=H, width=W, seed=43, device=gpu)
    cfg, ds = DecoderSplattingCUDACfg("splatting_cuda"), {"background_color": [0.1, 0.2, 0.3]}
    G = sc.gaussians.means.shape[1]
    ref_dec = DecoderSplattingCUDA(cfg, ds, seg_capacity=G).to(gpu)
    dec = DecoderSplattingCUDA(cfg, ds, seg_capacity=64).to(gpu)
    for d in (ref_dec, dec):
        d.raster_ctx.hints["max_count"] = 2048
        d.raster_ctx.adapt_hints = False

    def call(d):
        with torch.no_grad():
            return d(sc.gaussians, sc.target_extrinsics, sc.target_intrinsics, sc.near, sc.far, (H, W)).color

    want = call(ref_dec).clone()
    g = GraphedCall(lambda: call(dec), warmup=2)
    assert dec.raster_ctx.last_stats()["max_count"] > 64  # the frozen capacity overflows
    for _ in range(3):
        got = g()
        torch.cuda.synchronize()
        assert torch.equal(got, want)
