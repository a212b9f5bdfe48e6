#!/usr/bin/env python
"""Benchmark: rendered target views/sec on the reference's headline workload.

Workload (BASELINE.json configs[1]): RE10K-shaped 2-view 256x256 context -> 1 Gaussian
per pixel (G = 131,072), fp32, rendered into v = 3 target views (the RE10K evaluation
index: 2 context, 3 target views per scene). One "step" = one DecoderSplattingCUDA
forward of one scene batch (B scenes x v views) with the Gaussians already resident in
HBM — the `decoder` timer of the reference test loop (model_wrapper.py:432-484).
Synthetic inputs through the Gaussian adapter (my_depthsplat_amd.synthetic).

N GPUs: one process per GPU (torchrun), each rank renders its own scenes (per-scene data
parallel, no collective on the data path) -> scaling "weak"; value = all views / max time.

Extra fields: roofline of the dominant kernel (HIP events around its launches on the
stream it runs on; algorithmic bytes per launch in DESIGN.md §4), cpu_baseline (the CPU
oracle on the host, rank 0, bounded sample), psnr_vs_oracle_db (parity PSNR of one view).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip-level table (spec); 6.29 TB/s measured copy


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=500)  # ~30 ms timed at ~60 us per scene
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--batch", type=int, default=1, help="scenes per step per GPU (reference test loop: 1)")
    p.add_argument("--views", type=int, default=3, help="target views per scene (RE10K eval: 3)")
    p.add_argument("--size", type=int, default=256)
    p.add_argument("--context", type=int, default=2)
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--eager", action="store_true", help="time eager launches only (no hipGraph capture)")
    p.add_argument("--launch", choices=["auto", "hipgraph", "eager"] + [f"hipgraph{n}" for n in range(2, 9)], default="auto",
                   help="launch mode of the timed region (auto: the fastest in a short calibration of all)")
    p.add_argument("--extra", default="train,dl3dv,recon12",
                   help="secondary measurements: train (config C step), dl3dv (6-view 448x768 render), "
                        "recon12 (12-view 512x960 reconstruction, 100 views in chunks of 10); '' = none")
    p.add_argument("--extra-steps", type=int, default=10)
    return p.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from my_depthsplat_amd import _lib, raster
    from my_depthsplat_amd.decoder import DecoderSplattingCUDA, DecoderSplattingCUDACfg
    from my_depthsplat_amd.synthetic import make_scene

    _lib.load()
    H = W = args.size
    sc = make_scene(batch=args.batch, n_context=args.context, n_targets=args.views, height=H, width=W,
                    seed=1000 + rank, device=dev)
    dec = DecoderSplattingCUDA(DecoderSplattingCUDACfg("splatting_cuda"), {"background_color": [0.0, 0.0, 0.0]}).to(dev)
    dec = dec.to(dev)

    def step():
        with torch.no_grad():
            return dec(sc.gaussians, sc.target_extrinsics, sc.target_intrinsics, sc.near, sc.far, (H, W))

    for _ in range(args.warmup):
        out = step()
    torch.cuda.synchronize()
    n_rendered = raster.last_stats()["num_rendered"]  # also primes the LDS-sort size hint
    # short eager pass timing every launch -> the dominant kernel
    probe = raster.KernelTimer()
    raster.set_timer(probe)
    for _ in range(max(3, args.warmup)):
        out = step()
    raster.set_timer(None)
    dominant = max(probe.summary().items(), key=lambda kv: kv[1][0] * kv[1][1])[0]
    all_kernels = probe.summary()

    def timed(fn, steps):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        return time.perf_counter() - t0

    # launch mode: the whole decoder call replayed as ONE hipGraph per step, or launched
    # eagerly (the host runs ahead of the device, so launch gaps hide either way; on the
    # MI355X boxes eager measured ~2 % faster: graph kernel nodes are separated by heavier
    # barriers). A short calibration of both picks the mode; every kernel runs in both.
    # "hipgraphN" (N = 2..4): N such graphs (own buffers each) replayed in turn on N HIP
    # streams, so consecutive scenes overlap — one scene's compositing tail shares the chip with the
    # next scene's binning. Every step still renders its whole scene; only the overlap differs.
    runner, mode, cal = step, "eager", None
    if not args.eager:
        from my_depthsplat_amd.graphs import GraphedCall
        graphed = GraphedCall(step, warmup=2)
        out = graphed()
        max_lanes = int(os.environ.get("DSPLAT_BENCH_MAX_LANES", "4"))
        graphs = [graphed] + [GraphedCall(step, warmup=2) for _ in range(max_lanes - 1)]
        lanes = [torch.cuda.Stream(device=dev) for _ in graphs]
        turn = [0]

        def multi_stream(n):
            def run():
                i = turn[0] % n
                turn[0] += 1
                with torch.cuda.stream(lanes[i]):
                    return graphs[i]()
            return run

        modes = {"hipgraph": graphed, **{f"hipgraph{n}": multi_stream(n) for n in range(2, max_lanes + 1)},
                 "eager": step}
        if args.launch == "auto":
            ncal = max(10, min(50, args.steps))
            cal = {m: timed(fn, ncal) for m, fn in modes.items()}
            if world > 1:  # every rank takes the same decision
                t = torch.tensor(list(cal.values()), device=dev, dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                cal = dict(zip(cal, t.tolist()))
            mode = min(cal, key=cal.get)
            cal = {m: round(1e3 * t / ncal, 4) for m, t in cal.items()}
        else:
            mode = args.launch
        runner = modes[mode]
    # timed region 1 (value): exactly K steps in the chosen mode
    elapsed = timed(runner, args.steps)
    if mode.startswith("hipgraph") and mode != "hipgraph":  # the captures in use rendered the same scene
        used = graphs[:int(mode[len("hipgraph"):])]
        assert all(torch.equal(graphed.out.color, g.out.color) for g in used), f"{mode} captures disagree"
    # timed region 2: the same K steps launched eagerly, with HIP events recorded around the
    # dominant kernel on its launch stream (its average duration feeds the roofline)
    ev = raster.KernelTimer(only=[dominant])
    raster.set_timer(ev)
    elapsed_eager = timed(step, args.steps)
    raster.set_timer(None)
    ktimes = ev.summary()  # name -> (launches, avg_ms)
    if world > 1:
        t = torch.tensor([elapsed, elapsed_eager], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, elapsed_eager = (float(x) for x in t.tolist())
    views_per_step = args.batch * args.views
    total_views = views_per_step * args.steps * world
    value = total_views / elapsed

    if rank == 0:
        G = sc.gaussians.means.shape[1]
        V = views_per_step
        HW = H * W
        # dominant kernel + its algorithmic bytes per launch
        name = dominant
        launches, avg_ms = ktimes[name]
        alg = raster.algorithmic_bytes(name, G=G, V=V, N=n_rendered, HW=HW)
        achieved = alg / (avg_ms * 1e-3) / 1e9
        traffic, traffic_src = pmc_traffic(name, f"{args.context}v{H}x{W}x{args.views}b{args.batch}")
        roof = {"bound": "hbm", "kernel": name, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                "traffic_source": traffic_src,
                "avg_ms": round(avg_ms, 5), "algorithmic_bytes_per_launch": alg,
                "launches_timed": launches,
                "per_kernel_avg_ms_probe": {k: round(v[1], 5) for k, v in sorted(all_kernels.items())},
                "valu_issue": pmc_valu(name, f"{args.context}v{H}x{W}x{args.views}b{args.batch}", avg_ms)}
        psnr, l1, cpu = None, None, None
        if not args.no_cpu_baseline:
            psnr, l1, cpu = cpu_leg(sc, out, args, H, W)
    extra = {}
    wanted = [e for e in args.extra.split(",") if e]
    if "train" in wanted:
        extra["train_config_c"] = train_leg(args, dev, rank, world, timed)
    if "dl3dv" in wanted:
        extra["render_config_d"] = dl3dv_leg(args, dev, rank, world, timed)
    if "recon12" in wanted:
        extra["recon_config_e"] = recon12_leg(args, dev, rank, world, timed)
    if rank == 0:
        line = {
            "metric": "rendered views/sec + PSNR, 2-view 256x256 RE10K, 1/2/4/8 MI355X",
            "value": round(value, 2), "unit": "views/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 4), "higher_is_better": True,
            "launch_mode": mode, "launch_calibration_ms_per_step": cal,
            "ms_per_step_eager": round(1e3 * elapsed_eager / args.steps, 4),
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"{args.context}-view {H}x{W} RE10K feed-forward render, 1 Gaussian/pixel "
                                   f"(G={G}), {args.views} target views/scene, fp32",
                       "global_batch": args.batch * world, "views_per_scene": args.views, "gaussians": G,
                       "num_rendered_per_step": n_rendered, "parallelism": f"dp{world} (per-scene, no collective)",
                       "scenes_in_flight_per_gpu": int(mode[len("hipgraph"):] or 1) if mode.startswith("hipgraph") else 1},
            "psnr_vs_oracle_db": psnr, "l1_vs_oracle": l1,
            "roofline": roof, "cpu_baseline": cpu,
            **extra,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def pmc_traffic(kernel, workload):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary of the same
    workload (profiles/pmc_traffic.json, written by tools/pmc_summary.py --json: FETCH_SIZE
    x2 per the gfx950 correction + WRITE_SIZE, separate --pmc passes). None if absent."""
    f = ROOT / "profiles" / "pmc_traffic.json"
    if not f.exists():
        return None, None
    d = json.loads(f.read_text())
    rec = _pmc_record(d, kernel)
    if d.get("workload") != workload or rec is None:
        return None, None
    return int(rec["hbm_bytes"]), f"profiles/pmc_traffic.json ({d.get('source', '')})"


def _pmc_record(d, kernel):
    """The PMC entry of `kernel` (template instantiations are listed as name<args>)."""
    ks = d.get("kernels", {})
    if kernel in ks:
        return ks[kernel]
    return next((v for k, v in ks.items() if k.startswith(kernel + "<")), None)


def pmc_valu(kernel, workload, avg_ms):
    """VALU issue rate of `kernel`: SQ_INSTS_VALU per launch (wave-level instructions, from
    the committed PMC summary of the same workload) over its live average duration, against
    the chip's issue peak (256 CUs x 4 SIMDs, a wave64 VALU instruction every 4 cycles of a
    16-lane SIMD at ~2.4 GHz: 614 G wave-instructions/s). The compositor is issue / latency
    bound, not HBM bound; this is its roofline on the resource that binds."""
    f = ROOT / "profiles" / "pmc_traffic.json"
    if not f.exists():
        return None
    d = json.loads(f.read_text())
    rec = _pmc_record(d, kernel)
    if d.get("workload") != workload or rec is None or "SQ_INSTS_VALU" not in rec:
        return None
    peak = 256 * 4 * 2.4e9 / 4 / 1e9  # G wave-instructions / s
    ach = rec["SQ_INSTS_VALU"] / (avg_ms * 1e-3) / 1e9
    return {"achieved": round(ach, 1), "peak": peak, "unit": "G wave-instr/s", "frac": round(ach / peak, 4),
            "valu_instr_per_launch": int(rec["SQ_INSTS_VALU"]), "source": "profiles/pmc_traffic.json"}


def train_leg(args, dev, rank, world, timed):
    """Config C (BASELINE.json configs[2]): 2-view 256x256, 16 scenes x 4 target views per
    step, Gaussians from the adapter (head outputs are the trainable leaf), rasterizer forward
    + backward of an L1 + MSE colour loss, SGD update of the head. Per GPU; weak scaling."""
    import torch

    from my_depthsplat_amd.decoder import DecoderSplattingCUDA, DecoderSplattingCUDACfg
    from my_depthsplat_amd.gaussian_adapter import GaussianAdapter, GaussianAdapterCfg, gaussians_from_head
    from my_depthsplat_amd.loss import l1_mse_loss
    from my_depthsplat_amd.synthetic import context_cameras, target_cameras

    B, V, v, H, W = 16, 2, 4, 256, 256
    g = torch.Generator(device=dev).manual_seed(77 + rank)
    adapter = GaussianAdapter(GaussianAdapterCfg(1e-10, 3.0, 2)).to(dev)
    head = torch.randn(B, V, H * W, 3 + adapter.d_in, generator=g, device=dev).requires_grad_(True)
    depths = torch.rand(B, V, H * W, 1, 1, generator=g, device=dev) * 9 + 1
    images = torch.rand(B, V, 3, H, W, generator=g, device=dev)
    gt = torch.rand(B, v, 3, H, W, generator=g, device=dev)
    ctx = context_cameras(V)[None].repeat(B, 1, 1, 1).to(dev)
    K = torch.tensor([[1.0, 0, 0.5], [0, 1.0, 0.5], [0, 0, 1]], device=dev)
    ctx_k = K.expand(B, V, 3, 3).contiguous()
    tgt = target_cameras(context_cameras(V), v)[None].repeat(B, 1, 1, 1).to(dev)
    tgt_k = K.expand(B, v, 3, 3).contiguous()
    near = torch.full((B, v), 0.5, device=dev)
    far = torch.full((B, v), 100.0, device=dev)
    dec = DecoderSplattingCUDA(DecoderSplattingCUDACfg("splatting_cuda"), {"background_color": [0.0, 0.0, 0.0]}).to(dev)

    def step():
        gs = gaussians_from_head(head, depths, images, ctx, ctx_k, adapter)
        color = dec(gs, tgt, tgt_k, near, far, (H, W)).color
        loss = l1_mse_loss(color, gt, 1.0, 1.0)  # fused loss + gradient (dls_l1_mse_psnr)
        loss.backward()
        with torch.no_grad():
            head.sub_(1e-3 * head.grad)
            head.grad = None
        return loss

    for _ in range(2):
        step()
    el = timed(step, args.extra_steps)
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
    ms = 1e3 * el / args.extra_steps
    return {"workload": "config C: 2-view 256x256, 16 scenes x 4 target views, adapter + raster fwd+bwd, "
                        "L1+MSE loss, SGD on head outputs (no encoder network: out of scope)",
            "ms_per_step": round(ms, 3), "views_per_s": round(B * v * world / (ms * 1e-3), 1), "steps": args.extra_steps,
            "n_gpus": world}


def dl3dv_leg(args, dev, rank, world, timed):
    """6-view 448x768 (north_star's second input), 1 Gaussian per pixel (G = 2,064,384),
    8 target views per scene, forward render through the decoder. Per GPU; weak scaling."""
    import torch

    from my_depthsplat_amd.decoder import DecoderSplattingCUDA, DecoderSplattingCUDACfg
    from my_depthsplat_amd.synthetic import make_scene

    H, W, v = 448, 768, 8
    sc = make_scene(batch=1, n_context=6, n_targets=v, height=H, width=W, seed=2000 + rank, device=dev)
    dec = DecoderSplattingCUDA(DecoderSplattingCUDACfg("splatting_cuda"), {"background_color": [0.0, 0.0, 0.0]}).to(dev)

    def step():
        with torch.no_grad():
            return dec(sc.gaussians, sc.target_extrinsics, sc.target_intrinsics, sc.near, sc.far, (H, W))

    for _ in range(2):
        step()
    el = timed(step, args.extra_steps)
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
    ms = 1e3 * el / args.extra_steps
    return {"workload": f"6-view {H}x{W} render, G={sc.gaussians.means.shape[1]}, {v} target views/scene, fp32",
            "ms_per_step": round(ms, 3), "views_per_s": round(v * world / (ms * 1e-3), 1), "steps": args.extra_steps,
            "n_gpus": world}


def recon12_leg(args, dev, rank, world, timed):
    """BASELINE.json configs[4]: 12-view 512x960 feed-forward reconstruction (G = 5,898,240
    Gaussians from the fused adapter), then 100 target views rendered in chunks of 10
    (render_chunk_size, README.md:198). One step = adapter + 10 decoder calls for one scene.
    The reference's 0.6 s per scene on an A100 (README.md:105) also includes the encoder
    network, which is out of scope here, so no ratio is reported. Per GPU; weak scaling."""
    import torch

    from my_depthsplat_amd.decoder import DecoderSplattingCUDA, DecoderSplattingCUDACfg
    from my_depthsplat_amd.gaussian_adapter import GaussianAdapter, GaussianAdapterCfg, gaussians_from_head
    from my_depthsplat_amd.synthetic import context_cameras, target_cameras

    V, H, W, v, chunk = 12, 512, 960, 100, 10
    g = torch.Generator(device=dev).manual_seed(99 + rank)
    adapter = GaussianAdapter(GaussianAdapterCfg(1e-10, 3.0, 2)).to(dev)
    head = torch.randn(1, V, H * W, 3 + adapter.d_in, generator=g, device=dev)
    depths = torch.rand(1, V, H * W, 1, 1, generator=g, device=dev) * 9 + 1
    images = torch.rand(1, V, 3, H, W, generator=g, device=dev)
    K = torch.tensor([[1.0, 0, 0.5], [0, 1.0, 0.5], [0, 0, 1]], device=dev)
    ctx = context_cameras(V)[None].to(dev)
    tgt = target_cameras(context_cameras(V), v)[None].to(dev)
    ctx_k, tgt_k = K.expand(1, V, 3, 3).contiguous(), K.expand(1, v, 3, 3).contiguous()
    near = torch.full((1, v), 0.5, device=dev)
    far = torch.full((1, v), 100.0, device=dev)
    dec = DecoderSplattingCUDA(DecoderSplattingCUDACfg("splatting_cuda"), {"background_color": [0.0, 0.0, 0.0]}).to(dev)
    out = torch.empty(1, v, 3, H, W, device=dev)

    def step():
        with torch.no_grad():
            gs = gaussians_from_head(head, depths, images, ctx, ctx_k, adapter)
            for c in range(0, v, chunk):
                sl = slice(c, min(v, c + chunk))
                out[:, sl] = dec(gs, tgt[:, sl], tgt_k[:, sl], near[:, sl], far[:, sl], (H, W)).color

    step()
    steps = max(2, args.extra_steps // 2)
    el = timed(step, steps)
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
    ms = 1e3 * el / steps
    return {"workload": f"{V}-view {H}x{W} reconstruction, G={V * H * W}, adapter + {v} target views in chunks of "
                        f"{chunk} (encoder network out of scope), fp32",
            "ms_per_scene": round(ms, 2), "views_per_s": round(v * world / (ms * 1e-3), 1), "steps": steps,
            "n_gpus": world, "reference": "0.6 s per scene end to end on an A100 incl. the encoder (README.md:105)"}


def cpu_leg(sc, out, args, H, W):
    """CPU oracle on the host: parity PSNR/L1 of view 0 + a bounded throughput sample."""
    import numpy as np
    import torch

    from my_depthsplat_amd.cuda_splatting import _cov6, camera_settings
    from oracle import raster as orc

    g = sc.gaussians
    st = camera_settings(sc.target_extrinsics[0].cpu(), sc.target_intrinsics[0].cpu(), sc.near[0].cpu(),
                         sc.far[0].cpu())
    npst = {k: t.numpy() for k, t in st.items()}
    means = g.means[0].cpu().numpy()
    shs = g.harmonics[0].transpose(-1, -2).contiguous().cpu().numpy()
    opac = g.opacities[0].cpu().numpy()
    cov6 = _cov6(g.covariances[0]).contiguous().cpu().numpy()
    bg = np.zeros(3, np.float32)
    deg = int(round(shs.shape[1] ** 0.5)) - 1

    def one(i):
        return orc.render_settings(means, shs, None, opac, cov6, npst, i, bg, H, W, deg)

    o = one(0)
    ref, _, _ = o.image()
    o.close()
    hip = out.color[0, 0].float().cpu().numpy()
    l1 = float(np.abs(hip - ref).mean())
    mse = float(np.mean((np.clip(hip, 0, 1) - np.clip(ref, 0, 1)) ** 2))
    psnr = None if mse == 0 else round(-10 * np.log10(mse), 3)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    n, t0 = 0, time.perf_counter()
    while True:
        o = one(n % args.views)
        o.close()
        n += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds and n >= 2:
            break
    return psnr, l1, {"value": round(n / el, 3), "unit": "views/s", "cores": threads, "kind": "port",
                      "sample": f"{n} target views of the same {H}x{W} scene (G={means.shape[0]}) rendered by "
                                f"oracle/dsr_oracle.cpp (OpenMP, {threads} threads) in {el:.1f}s"}


if __name__ == "__main__":
    main()
