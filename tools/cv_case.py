"""Run one cost-volume bench shape (bench._costvol_case) N times for rocprofv3 passes.
usage: python tools/cv_case.py TAG [N] [--bwd]   (config_d_* tags: the views API, as the bench)"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402
from my_depthsplat_amd.matching import plane_sweep_cost_volume, plane_sweep_cost_volume_views  # noqa: E402

tag = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 20
dev = torch.device("cuda:0")
ref, tgt, K, pose, depth, shape = bench._costvol_case(tag, dev, 0)
views = tag.startswith("config_d")  # bench's config-D cases: features once + the neighbour index
if "--bwd" in sys.argv:
    ref.requires_grad_(True)
    if not views:
        tgt.requires_grad_(True)
for _ in range(n):
    if views:
        c = plane_sweep_cost_volume_views(ref, tgt, K, pose, depth, max_fanin=shape[1])
    else:
        c = plane_sweep_cost_volume(ref, tgt, K, pose, depth)
    if "--bwd" in sys.argv:
        c.sum().backward()
torch.cuda.synchronize()
print(tag, shape, "ok")
