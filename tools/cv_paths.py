"""Time dcv_cost_volume_fwd / fwd + bwd with the band kernel and with the epipolar-group kernels
(DSPLAT_CV_PATH) on the bench's cost-volume shapes and a few grid sizes between them, to place
the band / epipolar threshold (dcv_cost_volume.hip: kBandMaxPixels). GPU box only.
usage: python tools/cv_paths.py [out.json]"""
import json
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from my_depthsplat_amd.matching import plane_sweep_cost_volume  # noqa: E402


def timed_ms(fn, n):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def two_view(BV, C, H, W, D, dev):
    g = torch.Generator(device=dev).manual_seed(5)
    K = torch.tensor([[W * 1.0, 0, W / 2], [0, H * 1.0, H / 2], [0, 0, 1]], device=dev).expand(BV, 1, 3, 3)
    pose = torch.eye(4, device=dev).repeat(BV, 1, 1, 1)
    pose[:, :, 0, 3] = 0.1
    depth = (1.0 / torch.linspace(1 / 0.5, 1 / 100.0, D, device=dev)).expand(BV, D).contiguous()
    ref = torch.randn(BV, C, H, W, generator=g, device=dev)
    tgt = torch.randn(BV, 1, C, H, W, generator=g, device=dev)
    return ref, tgt, K.contiguous(), pose, depth


def main():
    dev = torch.device("cuda:0")
    cases = {f"{tag}": bench._costvol_case(tag, dev, 0)[:5] for tag in
             ("config_a_32x32", "config_b_scale0_64x64", "config_d_scale0_56x96", "config_d_scale1_112x192")}
    for BV, H, W in ((4, 64, 64), (8, 64, 64), (2, 128, 128), (16, 64, 64)):
        cases[f"2view_b{BV}_{H}x{W}"] = two_view(BV, 128, H, W, 128, dev)
    res = {}
    for tag, (ref, tgt, K, pose, depth) in cases.items():
        ent = {"B_HW": ref.shape[0] * ref.shape[2] * ref.shape[3]}
        for path in ("band", "epi"):
            os.environ["DSPLAT_CV_PATH"] = path
            ms = timed_ms(lambda: plane_sweep_cost_volume(ref, tgt, K, pose, depth), 30)
            rg, tg_ = ref.clone().requires_grad_(True), tgt.clone().requires_grad_(True)
            dcost = torch.randn(ref.shape[0], depth.shape[1], ref.shape[2], ref.shape[3], device=dev)

            def fb():
                rg.grad = tg_.grad = None
                (plane_sweep_cost_volume(rg, tg_, K, pose, depth) * dcost).sum().backward()
            ms_fb = timed_ms(fb, 10)
            ent[path] = {"fwd_ms": round(ms, 5), "fwd_bwd_ms": round(ms_fb, 5)}
        os.environ.pop("DSPLAT_CV_PATH")
        ent["auto_fwd_ms"] = round(timed_ms(lambda: plane_sweep_cost_volume(ref, tgt, K, pose, depth), 30), 5)
        res[tag] = ent
        print(tag, json.dumps(ent), flush=True)
    if len(sys.argv) > 1:
        Path(sys.argv[1]).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
