"""Per-(view, tile) entry-count distribution of a synthetic scene (GPU box).
usage: python tools/segstats.py CONTEXT H W TARGETS"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from my_depthsplat_amd import raster  # noqa: E402
from my_depthsplat_amd.decoder import DecoderSplattingCUDA, DecoderSplattingCUDACfg  # noqa: E402
from my_depthsplat_amd.synthetic import make_scene  # noqa: E402

V, H, W, v = (int(x) for x in sys.argv[1:5])
dev = torch.device("cuda:0")
sc = make_scene(batch=1, n_context=V, n_targets=v, height=H, width=W, seed=2000, device=dev)
dec = DecoderSplattingCUDA(DecoderSplattingCUDACfg("splatting_cuda"), {"background_color": [0.0, 0.0, 0.0]}).to(dev)
with torch.no_grad():
    dec(sc.gaussians, sc.target_extrinsics, sc.target_intrinsics, sc.near, sc.far, (H, W))
torch.cuda.synchronize()
c = raster._last["counts"].cpu().numpy()
print(f"G={sc.gaussians.means.shape[1]} views={v} tiles/view={c.size // v} N={c.sum()} mean={c.mean():.0f} "
      f"p50={np.percentile(c, 50):.0f} p90={np.percentile(c, 90):.0f} p99={np.percentile(c, 99):.0f} max={c.max()} "
      f">4096: {(c > 4096).mean():.3f} >8192: {(c > 8192).mean():.3f} >16384: {(c > 16384).mean():.3f}")
