"""Config C training step (bench.py train leg) eager vs captured whole into one hipGraph
(forward, backward and the SGD update replayed as one graph), GPU box.
usage: python tools/train_graph_exp.py [steps]"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from my_depthsplat_amd.decoder import DecoderSplattingCUDA, DecoderSplattingCUDACfg  # noqa: E402
from my_depthsplat_amd.gaussian_adapter import GaussianAdapter, GaussianAdapterCfg, gaussians_from_head  # noqa: E402
from my_depthsplat_amd.graphs import GraphedCall  # noqa: E402
from my_depthsplat_amd.loss import l1_mse_loss  # noqa: E402
from my_depthsplat_amd.synthetic import context_cameras, target_cameras  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda:0")
B, V, v, H, W = 16, 2, 4, 256, 256
g = torch.Generator(device=dev).manual_seed(77)
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
    loss = l1_mse_loss(color, gt, 1.0, 1.0)
    loss.backward()
    with torch.no_grad():
        head.add_(head.grad, alpha=-1e-3)
        head.grad = None
    return loss.detach()


def timeit(fn, n):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


print(f"eager   {timeit(step, steps):7.3f} ms/step", flush=True)
h0 = head.detach().clone()
gc = GraphedCall(step, warmup=3)
print(f"graphed {timeit(gc, steps):7.3f} ms/step", flush=True)
# the replay must keep training: the head moves every replay and the loss is finite
l0 = float(gc())
h1 = head.detach().clone()
gc()
print(f"loss {l0:.5f}; head moved {float((head.detach() - h1).abs().max()):.3e} per replay; "
      f"total drift {float((head.detach() - h0).abs().max()):.3e}", flush=True)
