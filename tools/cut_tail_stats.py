"""Depth-cut tail statistics of one config-E chunk (bench.py recon12_leg's scene, first 10
target views): tiles flagged for the tail pass (a pixel still live after the written head),
their full list lengths and head lengths, per view. usage: python tools/cut_tail_stats.py"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from my_depthsplat_amd import raster  # noqa: E402
from my_depthsplat_amd.decoder import DecoderSplattingCUDA, DecoderSplattingCUDACfg  # noqa: E402
from my_depthsplat_amd.gaussian_adapter import GaussianAdapter, GaussianAdapterCfg, gaussians_from_head  # noqa: E402
from my_depthsplat_amd.synthetic import context_cameras, target_cameras  # noqa: E402

dev = torch.device("cuda:0")
V, H, W, v = 12, 512, 960, 10
g = torch.Generator(device=dev).manual_seed(99)
adapter = GaussianAdapter(GaussianAdapterCfg(1e-10, 3.0, 2)).to(dev)
head = torch.randn(1, V, H * W, 3 + adapter.d_in, generator=g, device=dev)
depths = torch.rand(1, V, H * W, 1, 1, generator=g, device=dev) * 9 + 1
images = torch.rand(1, V, 3, H, W, generator=g, device=dev)
K = torch.tensor([[1.0, 0, 0.5], [0, 1.0, 0.5], [0, 0, 1]], device=dev)
ctx = context_cameras(V)[None].to(dev)
tgt_all = target_cameras(context_cameras(V), 100)[None].to(dev)
ctx_k, tgt_k = K.expand(1, V, 3, 3).contiguous(), K.expand(1, v, 3, 3).contiguous()
chunk_arg = int(sys.argv[1]) if len(sys.argv) > 1 else -1
near = torch.full((1, v), 0.5, device=dev)
far = torch.full((1, v), 100.0, device=dev)
dec = DecoderSplattingCUDA(DecoderSplattingCUDACfg("splatting_cuda"), {"background_color": [0.0, 0.0, 0.0]}).to(dev)
states = []
orig = raster.forward_raw


def spy(*a, **k):
    out = orig(*a, **k)
    states.append(out[1])
    return out


raster.forward_raw = spy
with torch.no_grad():
    gs = gaussians_from_head(head, depths, images, ctx, ctx_k, adapter)
    for c in range(10):
        states.clear()
        tgt = tgt_all[:, c * v:(c + 1) * v]
        dec(gs, tgt, tgt_k, near, far, (H, W))
        torch.cuda.synchronize()
        st = states[-1]
        gx, gy = raster.tiles(H, W)
        T = gx * gy
        ov = st.seg_overflow
        if ov is None:
            print("chunk", c, "no tail pass")
            continue
        flags = ov[: v * T].cpu().bool()
        full = st.tile_count.cpu().long()
        line = f"chunk {c} flagged {int(flags.sum())} any {int(ov[v * T].item())}"
        if flags.any():
            f = full[flags]
            line += f" flagged full mean {float(f.float().mean()):.0f} max {int(f.max())}"
        print(line, flush=True)
