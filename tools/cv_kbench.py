"""Time dcv_cost_volume_fwd across library variants at tools/cv_bench.py's shapes (GPU box);
outputs are compared with the first variant. usage: python tools/cv_kbench.py SHAPES VARIANT...
SHAPES = comma list of a, b0, b1, d0; VARIANT = lib/variants/libdsplat_NAME.so or "main"."""
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

from my_depthsplat_amd import _lib  # noqa: E402

SHAPES = {"a": (2, 1, 128, 32, 32, 128, False), "b0": (2, 1, 128, 64, 64, 128, False),
          "b1": (2, 1, 64, 128, 128, 32, True), "d0": (6, 2, 128, 56, 96, 128, False)}
dev = torch.device("cuda:0")
_lib.load()
st = _lib.stream_of(dev)


def fn_of(name):
    path = _lib.LIB_PATH if name == "main" else ROOT / "my_depthsplat_amd/lib/variants" / f"libdsplat_{name}.so"
    f = ctypes.CDLL(str(path)).dcv_cost_volume_fwd
    f.restype, f.argtypes = _lib.SIGNATURES["dcv_cost_volume_fwd"]
    return f


fns = {n: fn_of(n) for n in sys.argv[2:]}
for shp in sys.argv[1].split(","):
    B, J, C, H, W, D, pp = SHAPES[shp]
    g = torch.Generator(device=dev).manual_seed(0)
    ref = torch.randn(B, C, H, W, generator=g, device=dev)
    tgt = torch.randn(B, J, C, H, W, generator=g, device=dev)
    K = torch.tensor([[W * 1.0, 0, W / 2], [0, H * 1.0, H / 2], [0, 0, 1]], device=dev).expand(B, J, 3, 3).contiguous()
    pose = torch.eye(4, device=dev).repeat(B, J, 1, 1)
    pose[..., 0, 3] = -0.1
    d = torch.linspace(0.5, 10, D, device=dev)
    depth = d[None, :, None, None].expand(B, D, H, W).contiguous() if pp else d[None].expand(B, D).contiguous()
    first = None
    flops = 2.0 * B * J * C * D * H * W
    for name, f in fns.items():
        cost = torch.zeros(B, D, H, W, device=dev)

        def call():
            assert f(B, J, C, H, W, D, int(pp), ref.data_ptr(), tgt.data_ptr(), K.data_ptr(), pose.data_ptr(),
                     depth.data_ptr(), 1e-3, None, cost.data_ptr(), st) == 0
        for _ in range(5):
            call()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(200):
            call()
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 200
        first = cost.clone() if first is None else first
        diff = float((cost - first).abs().max())
        print(f"{shp:3s} {name:>10s}  {ms * 1e3:8.2f} us  {flops / ms / 1e9:7.2f} TFLOP/s  "
              f"({flops / ms / 1e9 / 157.3:.3f} of 157.3)  maxdiff {diff:.3e}", flush=True)
