"""Digest of the headline render (and of a depth-cut render) for same-box variant checks:
sha256 of the fp32 colour bytes of B = 4 config-B scenes (inference fast path) and of one
6-view 448x768 scene (two-phase depth-cut path), so a variant library (DSPLAT_LIB) can be
checked bit-identical to main. usage: python tools/img_digest.py [--cut]"""
import hashlib
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from my_depthsplat_amd.decoder import DecoderSplattingCUDA, DecoderSplattingCUDACfg  # noqa: E402
from my_depthsplat_amd.synthetic import make_scene  # noqa: E402

dev = torch.device("cuda:0")
out = {}
cases = [("b4_256", dict(batch=4, n_context=2, n_targets=3, height=256, width=256, seed=11))]
if "--cut" in sys.argv:
    cases.append(("d1_448x768", dict(batch=1, n_context=6, n_targets=4, height=448, width=768, seed=12)))
for name, kw in cases:
    sc = make_scene(device=dev, **kw)
    dec = DecoderSplattingCUDA(DecoderSplattingCUDACfg("splatting_cuda"), {"background_color": [0, 0, 0]}).to(dev)
    with torch.no_grad():
        for _ in range(2):  # second call: adapted hints (the bench's steady state)
            col = dec(sc.gaussians, sc.target_extrinsics, sc.target_intrinsics, sc.near, sc.far,
                      (kw["height"], kw["width"])).color
    torch.cuda.synchronize()
    out[name] = hashlib.sha256(col.contiguous().cpu().numpy().tobytes()).hexdigest()[:16]
print(" ".join(f"{k}={v}" for k, v in out.items()))
