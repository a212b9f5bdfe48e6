"""Phase timing of k_cost_epi from the instrumented variant (tools/cv_epi_timing_build.py), on
one view (J = 1) of a bench cost-volume shape. usage: python tools/cv_epi_timing.py [shape]"""
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from my_depthsplat_amd import _lib  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "config_d_scale0_56x96"
dev = torch.device("cuda:0")
ref, tgt, K, pose, depth, (BV, J, C, H, W, D) = bench._costvol_case(tag, dev, 0)
tgt, K, pose = tgt[:, :1].contiguous(), K[:, :1].contiguous(), pose[:, :1].contiguous()
lib = ctypes.CDLL(str(ROOT / "my_depthsplat_amd/lib/variants/libdsplat_cvt.so"))
for fn, (res, args) in _lib.SIGNATURES.items():
    f = getattr(lib, fn)
    f.restype, f.argtypes = res, args
HW = H * W
ngroups = (HW + 15) // 16
ws = torch.empty(lib.dcv_cost_volume_workspace_size(BV, 1, C, H, W), dtype=torch.uint8, device=dev)
cost = torch.zeros(BV * D * HW + BV * ngroups * 8, dtype=torch.float32, device=dev)
pp = int(depth.dim() == 4)
st = _lib.stream_of(dev)
for _ in range(5):
    assert lib.dcv_cost_volume_fwd(BV, 1, C, H, W, D, pp, 1, ref.data_ptr(), tgt.data_ptr(), K.data_ptr(), pose.data_ptr(),
                                   depth.data_ptr(), 1e-3, ws.data_ptr(), cost.data_ptr(), st) == 0
torch.cuda.synchronize()
r = cost[BV * D * HW:].view(torch.int32).cpu().numpy().astype(np.int64).reshape(-1, 8) & 0xFFFFFFFF
r = r[r[:, 0] > 0]
t = r[:, :6]
base = t[:, 0].min()
us = lambda x: x * 0.01  # noqa: E731
q = lambda a: f"mean={a.mean():7.2f} p10={np.percentile(a, 10):7.2f} p50={np.percentile(a, 50):7.2f} " \
              f"p90={np.percentile(a, 90):7.2f} max={a.max():7.2f}"  # noqa: E731
print(f"{tag} (one view): {len(t)} workgroups, span {us(t[:, 5].max() - base):.2f} us")
for k, name in enumerate(["aref", "front", "gemm", "gather", "tail"]):
    print(f"{name:8s} {q(us(t[:, k + 1] - t[:, k]))}")
print(f"lifetime {q(us(t[:, 5] - t[:, 0]))}")
print(f"U        {q(r[:, 6].astype(float))}")
