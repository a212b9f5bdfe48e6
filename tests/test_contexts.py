"""Per-caller rasterizer state (no global mutable state; safe for concurrent
calls on different streams and devices). Each decoder owns a RasterContext: its options and
the hints its own calls learn (LDS sort class, depth-cut plan, zeroed-counter pool)."""
from __future__ import annotations

import pytest
import torch

from my_depthsplat_amd import raster


def test_context_options_and_defaults(monkeypatch):
    ctx = raster.RasterContext(exact_binning=False)
    assert ctx.opt("exact_binning") is False
    monkeypatch.setattr(raster, "SORT_PREFIX", 123)  # unset options follow the module default
    assert ctx.opt("sort_prefix") == 123
    ctx.set(sort_prefix=7)
    assert ctx.opt("sort_prefix") == 7 and raster.SORT_PREFIX == 123
    with pytest.raises(TypeError):
        raster.RasterContext(no_such_option=1)
    with pytest.raises(TypeError):
        ctx.set(bogus=True)
    assert raster.default_context("cuda:0") is raster.default_context("cuda:0")
    assert raster.default_context("cuda:0") is not raster.default_context("cuda:1")


def test_decoders_own_their_contexts():
    from my_depthsplat_amd.decoder import DecoderSplattingCUDA, DecoderSplattingCUDACfg
    a = DecoderSplattingCUDA(DecoderSplattingCUDACfg("splatting_cuda"), {"background_color": [0, 0, 0]})
    b = DecoderSplattingCUDA(DecoderSplattingCUDACfg("splatting_cuda"), {"background_color": [0, 0, 0]},
                             exact_binning=False)
    assert a.raster_ctx is not b.raster_ctx
    a.raster_ctx.hints["max_count"] = 3000
    assert b.raster_ctx.hints["max_count"] == 0
    assert a.raster_ctx.opt("exact_binning") is True and b.raster_ctx.opt("exact_binning") is False


@pytest.mark.gpu
def test_two_decoders_interleaved_on_two_streams(gpu):
    """Two decoders with different workloads (config-B-like 256x256 scenes; large-Gaussian
    128x224 scenes whose tile lists are ~10x longer) interleaved on two HIP streams reproduce
    their solo outputs bit for bit, and each keeps its own LDS-class hint."""
    from my_depthsplat_amd.decoder import DecoderSplattingCUDA, DecoderSplattingCUDACfg
    from my_depthsplat_amd.synthetic import make_scene
    cfg, ds = DecoderSplattingCUDACfg("splatting_cuda"), {"background_color": [0.0, 0.0, 0.0]}
    sa = make_scene(batch=2, n_context=2, n_targets=3, height=256, width=256, seed=51, device=gpu)
    sb = make_scene(batch=1, n_context=2, n_targets=4, height=128, width=224, seed=52, device=gpu)
    sb.gaussians.covariances = sb.gaussians.covariances * 30.0

    def run(dec, sc):
        with torch.no_grad():
            return dec(sc.gaussians, sc.target_extrinsics, sc.target_intrinsics, sc.near, sc.far,
                       sc.image_shape).color

    solo = {}
    for name, sc in (("a", sa), ("b", sb)):
        dec = DecoderSplattingCUDA(cfg, ds).to(gpu)
        for _ in range(3):  # the hints settle after the first calls
            out = run(dec, sc)
        torch.cuda.synchronize()
        solo[name] = (out.clone(), dec.raster_ctx.hints["max_count"])
    assert solo["a"][1] != solo["b"][1]  # the two workloads want different LDS classes
    da, db = DecoderSplattingCUDA(cfg, ds).to(gpu), DecoderSplattingCUDA(cfg, ds).to(gpu)
    s1, s2 = torch.cuda.Stream(device=gpu), torch.cuda.Stream(device=gpu)
    outs = {"a": [], "b": []}
    for _ in range(4):
        with torch.cuda.stream(s1):
            outs["a"].append(run(da, sa))
        with torch.cuda.stream(s2):
            outs["b"].append(run(db, sb))
    torch.cuda.synchronize()
    for name in ("a", "b"):
        for o in outs[name]:
            assert torch.equal(o, solo[name][0]), name
    assert da.raster_ctx.hints["max_count"] == solo["a"][1]
    assert db.raster_ctx.hints["max_count"] == solo["b"][1]


@pytest.mark.gpu
def test_render_and_cost_volume_from_two_host_threads(gpu):
    """SURVEY §8(b) concurrency clause: a decoder render and a plane-sweep cost volume issued
    from two host threads at once, each on its own HIP stream, reproduce their solo outputs
    bit for bit (the library keeps no unsynchronised global state: the dynamic-LDS opt-ins are
    per (kernel, device) under a mutex, the raster state lives in each decoder's context)."""
    import threading

    from my_depthsplat_amd.decoder import DecoderSplattingCUDA, DecoderSplattingCUDACfg
    from my_depthsplat_amd.matching import plane_sweep_cost_volume
    from my_depthsplat_amd.synthetic import make_scene
    from test_cost_volume import _rig_case

    sc = make_scene(batch=2, n_context=2, n_targets=3, height=256, width=256, seed=61, device=gpu)
    ref, tgt, K, pose, depth = (t.to(gpu) for t in _rig_case(False, C=128, H=56, W=96, D=128, seed=62))
    dec = DecoderSplattingCUDA(DecoderSplattingCUDACfg("splatting_cuda"), {"background_color": [0.0, 0.0, 0.0]}).to(gpu)

    def render():
        with torch.no_grad():
            return dec(sc.gaussians, sc.target_extrinsics, sc.target_intrinsics, sc.near, sc.far, sc.image_shape).color

    def cost():
        return plane_sweep_cost_volume(ref, tgt, K, pose, depth)

    for _ in range(3):
        solo_r = render()
    solo_c = cost()
    torch.cuda.synchronize()
    solo_r, solo_c = solo_r.clone(), solo_c.clone()
    start = threading.Barrier(2)
    outs, errs = {"r": [], "c": []}, []

    def worker(key, fn):
        try:
            s = torch.cuda.Stream(device=gpu)
            start.wait()
            with torch.cuda.stream(s):
                for _ in range(6):
                    outs[key].append(fn())
            s.synchronize()
        except Exception as e:  # surfaced below (a thread's exception would be lost)
            errs.append(e)

    th = [threading.Thread(target=worker, args=("r", render)), threading.Thread(target=worker, args=("c", cost))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errs, errs
    assert len(outs["r"]) == 6 and len(outs["c"]) == 6
    torch.cuda.synchronize()
    for o in outs["r"]:
        assert torch.equal(o, solo_r)
    for o in outs["c"]:
        assert torch.equal(o, solo_c)
