"""Diagnostic: determinism and layout dependence of the raster gradients on the faint
large-tile scene (tests/test_raster_gpu.py::test_depth_cut_matches_full_scatter)."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
import numpy as np
import torch
from my_depthsplat_amd import raster
from test_raster_gpu import _forward_backward, _large_tile_scene
from raster_cases import settings_for, oracle_views, flat_inputs

gpu = torch.device("cuda:0")
raster.KEY_BUDGET_BYTES = 0
raster.SORT_PREFIX = 0
sc = _large_tile_scene(constant_opacity=0.0045)
st = settings_for(sc)
res = {}
for cutp in (1024, 0, 1024, 0):
    raster._spec["two_phase_max"] = None
    raster.CUT_PREFIX = cutp
    _, outs = _forward_backward(sc, st, gpu)
    res.setdefault(cutp, []).append(outs)
names = ["color", "T", "nc", "dmeans", "dshs", "dopac", "dcov6", "dm2d"]
for i in range(3, len(res[0][0])):
    a0, a1, b0, b1 = res[1024][0][i], res[1024][1][i], res[0][0][i], res[0][1][i]
    m = float(b0.abs().max())
    print(f"{names[i] if i < len(names) else i}: max {m:.3e} rep_cut {float((a0-a1).abs().max()):.3e} "
          f"rep_full {float((b0-b1).abs().max()):.3e} cut_vs_full {float((a0-b0).abs().max()):.3e}", flush=True)
# vs the oracle's backward (dmeans summed over views with the scale factor)
dcolor = torch.linspace(-1, 1, res[0][0][0].numel()).view_as(res[0][0][0])
acc = 0
for i, o in enumerate(oracle_views(sc, st)):
    gr = o.backward(dcolor[i].numpy())
    acc = acc + gr["dmean3D"] * float(st["scale"][i])
    o.close()
ref = np.asarray(acc)
for cutp in (1024, 0):
    h = res[cutp][0][3][0].numpy().reshape(ref.shape)
    print(f"cut {cutp}: dmeans vs oracle max err {np.abs(h - ref).max():.3e} (max {np.abs(ref).max():.3e})", flush=True)
