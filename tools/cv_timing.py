"""Phase timing of k_cost_band from an instrumented variant (GPU box): per workgroup,
s_memrealtime (100 MHz) at start, after the taps' box reduction (camera, sample geometry),
after the correlation GEMM (B loads + MFMA + LDS store), after the bilinear gather and at the
end (cost stores), written after the cost volume in an enlarged output buffer.
usage: python tools/cv_timing.py VARIANT [shape]   (shape as tools/cv_bench.py: a, b0, b1, d0)"""
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from my_depthsplat_amd import _lib  # noqa: E402

name = sys.argv[1]
shp = sys.argv[2] if len(sys.argv) > 2 else "b0"
SHAPES = {"a": (2, 1, 128, 32, 32, 128, False), "b0": (2, 1, 128, 64, 64, 128, False),
          "b1": (2, 1, 64, 128, 128, 32, True), "d0": (6, 2, 128, 56, 96, 128, False)}
B, J, C, H, W, D, pp = SHAPES[shp]
dev = torch.device("cuda:0")
_lib.load()
g = torch.Generator(device=dev).manual_seed(0)
ref = torch.randn(B, C, H, W, generator=g, device=dev)
tgt = torch.randn(B, J, C, H, W, generator=g, device=dev)
K = torch.tensor([[W * 1.0, 0, W / 2], [0, H * 1.0, H / 2], [0, 0, 1]], device=dev).expand(B, J, 3, 3).contiguous()
pose = torch.eye(4, device=dev).repeat(B, J, 1, 1)
pose[..., 0, 3] = -0.1
d = torch.linspace(0.5, 10, D, device=dev)
depth = d[None, :, None, None].expand(B, D, H, W).contiguous() if pp else d[None].expand(B, D).contiguous()
nwg = ((W + 15) // 16) * H * B * ((D + 63) // 64)
cost = torch.zeros(B * D * H * W + nwg * 16, device=dev)
lib = ctypes.CDLL(str(ROOT / "my_depthsplat_amd/lib/variants" / f"libdsplat_{name}.so"))
f = lib.dcv_cost_volume_fwd
f.restype, f.argtypes = _lib.SIGNATURES["dcv_cost_volume_fwd"]
st = _lib.stream_of(dev)
for _ in range(10):
    assert f(B, J, C, H, W, D, int(pp), ref.data_ptr(), tgt.data_ptr(), K.data_ptr(), pose.data_ptr(),
             depth.data_ptr(), 1e-3, None, cost.data_ptr(), st) == 0
torch.cuda.synchronize()
t = cost[B * D * H * W:].view(torch.int64).view(nwg, 8).cpu().numpy()
base = t[:, 0].min()
us = lambda x: x * 0.01  # noqa: E731
q = lambda a: f"mean={a.mean():6.2f} p10={np.percentile(a, 10):6.2f} p50={np.percentile(a, 50):6.2f} " \
              f"p90={np.percentile(a, 90):6.2f} max={a.max():6.2f}"  # noqa: E731
print(f"{name} {shp}: {nwg} workgroups, span {us(t[:, 4].max() - base):.2f} us")
print(f"start        {q(us(t[:, 0] - base))}")
print(f"geometry+box {q(us(t[:, 1] - t[:, 0]))}")
print(f"corr GEMM    {q(us(t[:, 2] - t[:, 1]))}")
print(f"gather       {q(us(t[:, 3] - t[:, 2]))}")
print(f"store        {q(us(t[:, 4] - t[:, 3]))}")
print(f"end          {q(us(t[:, 4] - base))}")
