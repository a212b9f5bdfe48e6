"""Forward / forward+backward time of one bench cost-volume shape on cuda:0 with the library
DSPLAT_LIB points at (variant experiments). usage: python tools/cv_fwd.py TAG [LABEL]"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402
from my_depthsplat_amd.matching import plane_sweep_cost_volume  # noqa: E402

tag = sys.argv[1]
label = sys.argv[2] if len(sys.argv) > 2 else ""
dev = torch.device("cuda:0")
ref, tgt, K, pose, depth, shape = bench._costvol_case(tag, dev, 0)


def timed(fn, n):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


fwd = timed(lambda: plane_sweep_cost_volume(ref, tgt, K, pose, depth), 30)
rg, tg_ = ref.clone().requires_grad_(True), tgt.clone().requires_grad_(True)
dc = torch.randn(shape[0], shape[5], shape[3], shape[4], device=dev)


def fb():
    rg.grad = tg_.grad = None
    (plane_sweep_cost_volume(rg, tg_, K, pose, depth) * dc).sum().backward()


print(f"{label:12s} {tag}: fwd {fwd:8.1f} us  fwd+bwd {timed(fb, 10):8.1f} us")
